#!/bin/bash
# rocprofv3 passes for the judged profile: kernel trace + stats, then one PMC pass per TCC counter
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).  Outputs under gpurun_out/prof_*.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS=${ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline"}
step() { local name=$1; shift; timeout -k 10 600 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
step prof_trace rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python bench.py $ARGS
step prof_fetch rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python bench.py $ARGS --no-stats
step prof_write rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python bench.py $ARGS --no-stats
step prof_sq rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/prof_sq -o run --output-format csv -- python bench.py $ARGS --no-stats
step prof_sq2 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU -d gpurun_out/prof_sq2 -o run --output-format csv -- python bench.py $ARGS --no-stats
step prof_sq3 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES -d gpurun_out/prof_sq3 -o run --output-format csv -- python bench.py $ARGS --no-stats
grep -h "render" gpurun_out/prof_trace/run_kernel_stats.csv
