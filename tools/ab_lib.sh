# A/B of the working library against libvaesne_hip_ab0.so (the previous build) and, if
# present, libvaesne_hip_ab1.so (an intermediate one): kernel parity of the decoder tails /
# attention first, then interleaved step timing
mkdir -p gpurun_out
L=/root/repo/vaesne-dev_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_rep_attention.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ab.log 2>&1 || exit $?
V=("VAESNE_HIP_LIB=$L/libvaesne_hip_ab0.so")
[ -f $L/libvaesne_hip_ab1.so ] && V+=("VAESNE_HIP_LIB=$L/libvaesne_hip_ab1.so")
V+=("VAESNE_HIP_LIB=$L/libvaesne_hip.so")
bash profiles/ab_env.sh "${V[@]}" > gpurun_out/ab_lib.txt 2>&1
