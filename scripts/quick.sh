#!/bin/bash
# GPU iteration: parity tests, then bench A/B lines from scripts/ab_list.txt (or $AB_LIST).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?
tail -3 gpurun_out/tests.log
echo "tests rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
bash scripts/ab_env.sh < "${AB_LIST:?set AB_LIST to a file of A/B lines (scripts/ab_env.sh)}"
