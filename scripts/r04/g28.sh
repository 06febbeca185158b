#!/bin/bash
# round-4: strong-scaling estimates of the final build (scripts/diag_scale.py: every rank's share on
# one GPU, gather modelled) for C2, C4 and C5, and the default bench line with the committed PMC roofline
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_check.log 2>&1; rc=$?; echo bench rc=$rc; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u scripts/diag_scale.py > gpurun_out/scale_c2.log 2>&1; rc=$?; echo c2 rc=$rc; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u scripts/diag_scale.py final 3840 2159 4 4 > gpurun_out/scale_c5.log 2>&1; rc=$?; echo c5 rc=$rc; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u scripts/diag_scale.py door 1920 1079 16 16 > gpurun_out/scale_c4.log 2>&1; rc=$?; echo c4 rc=$rc; [ $rc = 0 ] || exit $rc
