#!/bin/bash
# r06 session 20: two-kernel tail backward with weight-gradient chunks of up to 4 data chunks:
# tail tests, B = 2 step stamps A/B vs m16
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_determinism.py -q -rf --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/s20_tests.log 2>&1; rc=$?
tail -2 gpurun_out/s20_tests.log; [ $rc -le 1 ] || exit $rc
grep -qsE "illegal memory access|Memory access fault|HSA_STATUS_ERROR" gpurun_out/s20_tests.log && exit 3
for rep in 1 2; do
  for V in cur m16; do
    env=""; [ $V != cur ] && env="VAESNE_PKG_DIR=$PWD/abpkg/$V VAESNE_HIP_LIB=$PWD/abpkg/$V/libvaesne_hip.so"
    env $env VAESNE_STAMPS=1 timeout -k 10 300 python tools/stamps.py --batch 2 > gpurun_out/s20_b2_$V.txt 2>/dev/null || exit 5
    echo "$V $(grep -E '^update' gpurun_out/s20_b2_$V.txt)"
  done
done
