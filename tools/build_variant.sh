#!/bin/bash
# Build the current sources as an experiment variant of libxalm_hip.so:
#   tools/build_variant.sh NAME [extra hipcc flags]  ->  xalm_amd/lib/var_NAME.so
# Run it with XALM_HIP_LIB=xalm_amd/lib/var_NAME.so (xalm_amd/_lib.py).
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
obj=/tmp/xalm_var_$name
make -j8 OBJ=$obj LIB=$obj/lib HIPFLAGS_EXTRA="$*" $obj/lib/libxalm_hip.so > $obj.log 2>&1 || { tail -20 $obj.log; exit 1; }
cp $obj/lib/libxalm_hip.so xalm_amd/lib/var_$name.so
echo "xalm_amd/lib/var_$name.so"
