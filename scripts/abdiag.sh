set -u
for v in ${VARS:-D1}; do echo "== $v"; RT_HIP_LIB=build/ab/lib$v.so timeout -k 10 120 python scripts/diag_parity.py big1 96 54 2 3 || exit 1; done
