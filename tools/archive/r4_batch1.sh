mkdir -p gpurun_out
timeout -k 10 400 tools/ab_tb3_abl.sh 3 abl0 abl4 abl5 abl6 > gpurun_out/abl_mem.log 2>&1
echo "abl rc=$?"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_r4a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gputest_r4a.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 tools/archive/r4_fp32_scheme.sh > gpurun_out/fp32_scheme_r4.log 2>&1; echo "fp32 rc=$?"
cat gpurun_out/abl_mem.log gpurun_out/fp32_scheme_r4.log
