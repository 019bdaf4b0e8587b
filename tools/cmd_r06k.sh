export TMPDIR=/tmp
LIBS="base gqbal gqbal8" WL="mistral-7b-f8 mistral-7b-q8_0 mistral-7b-q4_0" ROUNDS=2 bash tools/gpu_step.sh ab9 900 bash tools/abn.sh
