# round 6: lean BB refinements A/B (next-group U/dx prefetch; W1 image row skew) against variants without
# each: gradient + fuzz tests of the product library first, then tools/time_bwd.py interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_grad.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06h_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r06h_pytest.log; [ $rc -ne 0 ] && exit $rc
ABL_LIBS="build_ab/lib_nopf.so build_ab/lib_noskew.so build_ab/lib_nolean.so" ABL_SIZES=1024x72,128x72 bash tools/r06_bb_abl.sh
