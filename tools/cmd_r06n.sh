export TMPDIR=/tmp
STEPS=64 LIBS="base s192 s224" WL="mistral-7b-f16-32k" ROUNDS=2 bash tools/gpu_step.sh ab11 900 bash tools/abn.sh
