#!/bin/bash
# Print value and kernel ms of the A/B bench logs named on the command line (gpurun_out/ab_NAME.log).
for f in "$@"; do
  python -c "
import json, sys
ls = [x for x in open('gpurun_out/ab_$f.log') if x.startswith('{')]
d = json.loads(ls[-1]) if ls else {}
print('$f', d.get('value'), d.get('kernel_ms'), d.get('cold_kernel_ms'))"
done
