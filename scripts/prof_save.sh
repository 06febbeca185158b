#!/bin/bash
# After scripts/prof_all.sh ran on the GPU box (gpurun_out/c{2..5}_*): write the PMC summaries and
# kernel stats of the four bench workloads into profiles/$1.  The profiled kernel of each workload is
# the render instantiation with the most dispatches in its trace (the timed draws; the counting
# pass of bench.py is a single dispatch of another instantiation).
set -e
R=${1:-r04}
cd "$(dirname "$0")/.."
mkdir -p profiles/$R
for c in c2 c3 c4 c5; do for k in trace fetch write sq sq2 sq3 l2; do
  [ -d gpurun_out/${c}_$k ] || { echo "missing gpurun_out/${c}_$k: run scripts/prof_all.sh on the GPU box first"; exit 1; }
done; done
kernel_of() {  # render_kernel<MASK> / render_step_kernel<MASK> with the most calls
  python - "$1" <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(f"gpurun_out/{sys.argv[1]}_trace/**/*kernel_stats.csv", recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if "render" in r["Name"]]
best = max(rows, key=lambda r: int(r["Calls"]))
print(best["Name"].split("::", 1)[1].split("(", 1)[0])
PY
}
W="10 fb x 10 spp = 100 rays/pixel, depth 50, cam ref, traversal culled"
PMC_LAST=2 python scripts/pmc_summary.py profiles/$R/c2_render_pmc.json "$(kernel_of c2)" "C2 big1 1200x800, $W" c2 > /dev/null
PMC_LAST=2 python scripts/pmc_summary.py profiles/$R/c3_render_pmc.json "$(kernel_of c3)" "C3 cornell_smoke 800x800, $W" c3 > /dev/null
PMC_LAST=2 python scripts/pmc_summary.py profiles/$R/c4_render_pmc.json "$(kernel_of c4)" "C4 door 1920x1079, 16 fb x 16 spp = 256 rays/pixel, depth 50, cam ref, traversal culled" c4 > /dev/null
PMC_LAST=2 python scripts/pmc_summary.py profiles/$R/c5_render_pmc.json "$(kernel_of c5)" "C5 final 3840x2159, 4 fb x 4 spp = 16 rays/pixel, depth 50, cam ref, traversal culled" c5 > /dev/null
for c in c2 c3 c4 c5; do cp gpurun_out/${c}_trace/run_kernel_stats.csv profiles/$R/${c}_kernel_stats.csv; done
