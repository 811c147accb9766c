# r03: block-1 attention backward over the copies' summed masked dO (G = sum_c keep_c dO_c)
# against the committed library (ab0), plus the forward-only geometry 256 x 1
mkdir -p gpurun_out
L=/root/repo/vaesne-dev_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_rep_attention.py tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_rep.log 2>&1 || exit $?
for G in 256,2 256,1 128,1; do
  VAESNE_ATTN_FWD_GEO=$G timeout -k 10 120 python bench.py --roofline-only > gpurun_out/rl_$G.json 2> gpurun_out/rl_$G.err || exit 5
done
bash profiles/ab_env.sh "VAESNE_HIP_LIB=$L/libvaesne_hip_ab0.so" "VAESNE_HIP_LIB=$L/libvaesne_hip.so" "VAESNE_ATTN_FWD_GEO=256,1" > gpurun_out/ab_rep.txt 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --throughput-batch 0 --no-extras > gpurun_out/prof_r.log 2>&1
