export TMPDIR=/tmp
for v in nogran gran; do for w in mistral-7b-f16 mistral-7b-f8; do
XALM_HIP_LIB=xalm_amd/lib/var_$v.so bash tools/gpu_step.sh trace_${v}_$w 200 python3 tools/aw_trace.py --workload $w || exit 1
done; done
