cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python tools/dbg/rep_bwd_dbg.py > gpurun_out/dbg.log 2>&1; tail -14 gpurun_out/dbg.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_rep_sf16.py tests/test_gpu_determinism.py tests/test_gpu_rep_attention.py -v -rf --maxfail=6 --timeout 300 --timeout-method thread > gpurun_out/s2_tests.log 2>&1; rc=$?
tail -15 gpurun_out/s2_tests.log; exit $rc
