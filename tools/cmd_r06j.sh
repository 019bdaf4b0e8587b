export TMPDIR=/tmp
LIBS="base bal" WL="mistral-7b-f16 mistral-7b-f8 mistral-7b-q4_0" ROUNDS=2 bash tools/gpu_step.sh ab8 900 bash tools/abn.sh
