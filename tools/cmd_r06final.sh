export TMPDIR=/tmp
bash tools/cmd_r06i.sh && SKIP_TESTS=1 PART=b ROUND=r06 bash tools/round_profiles.sh
