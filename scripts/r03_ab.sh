#!/bin/bash
# GPU session: parity suite on the tree's library, the mesh parity tests on an experiment library
# ($EXP_LIB), then the A/B bench lines of $AB_LIST.  Stops at the first crash-like exit.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -2 gpurun_out/tests.log; echo "tests rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
if [ -n "${EXP_LIB:-}" ]; then
  RT_HIP_LIB=$EXP_LIB timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "${EXP_K:-door or mesh or triangle or final}" > gpurun_out/tests_exp.log 2>&1
  rc=$?; tail -2 gpurun_out/tests_exp.log; echo "exp tests rc=$rc"
  case $rc in 0|1) ;; *) exit $rc;; esac
fi
bash scripts/ab_env.sh < ${AB_LIST:-scripts/ab_list.txt}
