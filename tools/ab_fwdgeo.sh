# forward-only attention geometry (VAESNE_ATTN_FWD_GEO): 256 x 2 (3 waves / SIMD at 164
# VGPRs: 4096 waves run as 1.33 rounds) against 256 x 1 / 128 x 1 (98 VGPRs, 4 waves / SIMD:
# 8192 waves = 2 full rounds, 2 queries per lane); parity of the tail changes first
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_rep_attention.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_geo.log 2>&1 || exit $?
for G in 256,2 256,1 128,1; do
  VAESNE_ATTN_FWD_GEO=$G timeout -k 10 120 python bench.py --roofline-only > gpurun_out/rl_$G.json 2> gpurun_out/rl_$G.err || exit 5
done
bash profiles/ab_env.sh "VAESNE_ATTN_FWD_GEO=256,2" "VAESNE_ATTN_FWD_GEO=256,1" "VAESNE_ATTN_FWD_GEO=128,1" > gpurun_out/ab_fwdgeo.txt 2>&1
