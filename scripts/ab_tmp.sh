# Env-knob sweep of the warm schedule (diag_split.py default thresholds): long prefix priority,
# cost bucket width, camera-list share rule.
set -e
run() { echo "== $*"; env "$@" DIAG_N=1,2,4,8 timeout -k 10 300 python scripts/diag_split.py 10 10 default default 2>/dev/null | grep warm; env "$@" DIAG_N=1,8 timeout -k 10 300 python scripts/diag_split.py 100 1 default default 2>/dev/null | grep warm; }
run RT_NONE=1
run RT_LONG_PCT=0
run RT_LONG_PCT=5
run RT_COST_SHIFT=2
run RT_COST_SHIFT=4
run RT_BINS_MIN_ITEMS_PER_LANE=0
