# A/B of the XCD-aware workgroup remap (libvaesne_hip_ab0.so = before): attention parity,
# roofline launches, step time, and the FETCH_SIZE pass of the new library.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_rep_attention.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_xcd.log 2>&1 || exit $?
for L in libvaesne_hip_ab0 libvaesne_hip; do
  VAESNE_HIP_LIB=/root/repo/vaesne-dev_amd/lib/$L.so timeout -k 10 120 python bench.py --roofline-only > gpurun_out/rl_$L.json 2> gpurun_out/rl_$L.err || exit 5
done
bash profiles/ab_env.sh "VAESNE_HIP_LIB=/root/repo/vaesne-dev_amd/lib/libvaesne_hip_ab0.so" "VAESNE_HIP_LIB=/root/repo/vaesne-dev_amd/lib/libvaesne_hip.so" > gpurun_out/ab_xcd.txt 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_x -o run --output-format csv -- python bench.py --roofline-only > gpurun_out/pmc_fetch_x.log 2>&1 || exit 7
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_x -o run --output-format csv -- python bench.py --roofline-only > gpurun_out/pmc_write_x.log 2>&1
