mkdir -p gpurun_out
VAESNE_SPEC_FIRST=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_specfirst.log 2>&1 || exit $?
bash profiles/ab_env.sh VAESNE_SPEC_FIRST=0 VAESNE_SPEC_FIRST=1 > gpurun_out/ab_specfirst.txt 2>&1
