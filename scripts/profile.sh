#!/bin/bash
# rocprofv3 passes for one bench workload: kernel trace + stats, then one PMC pass per counter
# group (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950; each pass its own run, never
# combined with any trace domain).  Outputs under gpurun_out/${NAME}_*.
#   NAME=c2 ARGS="--steps 2 --warmup 1 --no-cpu-baseline" bash scripts/profile.sh
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
NAME=${NAME:-c2}
ARGS=${ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline"}
step() { local name=$1; shift; timeout -k 10 ${STEP_TIMEOUT:-300} "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac; }
P="-d gpurun_out/${NAME}"
step ${NAME}_trace rocprofv3 --kernel-trace --stats -d gpurun_out/${NAME}_trace -o run --output-format csv -- python bench.py $ARGS
step ${NAME}_fetch rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${NAME}_fetch -o run --output-format csv -- python bench.py $ARGS --no-stats
step ${NAME}_write rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${NAME}_write -o run --output-format csv -- python bench.py $ARGS --no-stats
step ${NAME}_sq rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/${NAME}_sq -o run --output-format csv -- python bench.py $ARGS --no-stats
step ${NAME}_sq2 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_SMEM -d gpurun_out/${NAME}_sq2 -o run --output-format csv -- python bench.py $ARGS --no-stats
step ${NAME}_sq3 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES -d gpurun_out/${NAME}_sq3 -o run --output-format csv -- python bench.py $ARGS --no-stats
step ${NAME}_l2 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/${NAME}_l2 -o run --output-format csv -- python bench.py $ARGS --no-stats
grep -h "render" gpurun_out/${NAME}_trace/run_kernel_stats.csv
