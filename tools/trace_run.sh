set -u
cd $GRAFT_REPO_ROOT
for w in mistral-7b-f16 mistral-7b-f8; do for f in 1 2; do
  echo "=== $w fuse $f"; timeout -k 10 200 python tools/aw_trace.py --workload $w --fuse $f 2>&1 | grep -v amdgpu.ids || exit $?
done; done
