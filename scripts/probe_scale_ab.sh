#!/bin/bash
# diag_scale.py (C2 10 x 10 and C4) under several librt_hip.so builds and options:
#   bash scripts/probe_scale_ab.sh name=lib[@opt] ...
set -u
mkdir -p gpurun_out
for pair in "$@"; do
  name=${pair%%=*}; rest=${pair#*=}; lib=${rest%%@*}; opt=""
  case $rest in *@*) opt="--opt ${rest#*@}";; esac
  for sc in "big1 1200 800 10 10" ${PROBE_C4:+"door 1920 1079 16 16"}; do
    tag=$(echo $sc | cut -d' ' -f1)
    RT_HIP_LIB=$lib timeout -k 10 400 python -u scripts/diag_scale.py $sc $opt > gpurun_out/psc_${name}_$tag.txt 2>&1 || exit $?
    echo "$name $tag: $(grep '^N=' gpurun_out/psc_${name}_$tag.txt | sed 's/.*warm \([0-9.]*\) \/ cold \([0-9.]*\) ms + init.*/\1|\2/' | tr '\n' ' ')"
  done
done
