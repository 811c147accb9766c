# r03: decoder-tail fused backward (bit-arithmetic keep scales, zeroed gradients past the
# sequence end instead of per-store masks, exact context count in the forward tail) and
# the XCD-aware attention workgroup remap.  ab0 = before both, ab1 = remap only.
mkdir -p gpurun_out
L=/root/repo/vaesne-dev_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_rep_attention.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_tail.log 2>&1 || exit $?
bash profiles/ab_env.sh "VAESNE_HIP_LIB=$L/libvaesne_hip_ab0.so" "VAESNE_HIP_LIB=$L/libvaesne_hip_ab1.so" "VAESNE_HIP_LIB=$L/libvaesne_hip.so" > gpurun_out/ab_tail.txt 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_t -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --throughput-batch 0 --no-extras > gpurun_out/prof_t.log 2>&1
