# round-4: C5 occupancy A/B, C3 split A/B, C5 phase shares
export TMPDIR=/tmp; mkdir -p gpurun_out
cat > /tmp/ab.txt <<'AB'
c5w4 --scene final --width 3840 --height 2159 --spp 4 --nfb 4
c5w3 RT_HIP_LIB=build/ab/libwpe3.so --scene final --width 3840 --height 2159 --spp 4 --nfb 4
c3split --scene cornell_smoke --width 800 --height 800
c3nosplit RT_SPLIT_MIN_SEGMENTS=1e9 --scene cornell_smoke --width 800 --height 800
AB
bash scripts/ab_env.sh < /tmp/ab.txt || exit $?
RT_HIP_LIB=build/ab/libstamps.so timeout -k 10 120 python scripts/diag_stamps.py final 1280 720 8 8 > gpurun_out/stamps_c5.log 2>&1; echo stamps rc=$?
cat gpurun_out/stamps_c5.log
