#!/bin/bash
# column-form experiments: XALM_AC_DEBUG 0 (real), 1 (no attention), 2 (no Wo loads), 3 (neither)
for d in ${@:-0 1 2 3}; do
  echo "== XALM_AC_DEBUG=$d"
  XALM_AC_DEBUG=$d timeout -k 10 120 python -u tools/col_sweep.py || exit 1
done
