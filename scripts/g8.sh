# round-4 tuning A/B: render_kernel refill threshold (C5, C3), shading threshold of C4's quantized-LDS variant
export TMPDIR=/tmp; mkdir -p gpurun_out
cat > /tmp/ab.txt <<'AB'
c5r16 --scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats
c5r8 RT_HIP_LIB=build/ab/librefill8.so --scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats
c5r24 RT_HIP_LIB=build/ab/librefill24.so --scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats
c5r32 RT_HIP_LIB=build/ab/librefill32.so --scene final --width 3840 --height 2159 --spp 4 --nfb 4 --no-stats
c3r16 --scene cornell_smoke --width 800 --height 800 --no-stats
c3r8 RT_HIP_LIB=build/ab/librefill8.so --scene cornell_smoke --width 800 --height 800 --no-stats
c3r32 RT_HIP_LIB=build/ab/librefill32.so --scene cornell_smoke --width 800 --height 800 --no-stats
c4s48 --scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-stats
c4s40 RT_SHADE_MIN=40 --scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-stats
c4s56 RT_SHADE_MIN=56 --scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-stats
c4s60 RT_SHADE_MIN=60 --scene door --width 1920 --height 1079 --spp 16 --nfb 16 --no-stats
AB
bash scripts/ab_env.sh < /tmp/ab.txt || exit $?
