cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_window.py -x -q -p no:cacheprovider > gpurun_out/win_tests.log 2>&1; rc=$?
echo "window tests rc=$rc"; tail -3 gpurun_out/win_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/phase_probe.py || exit $?
CFGS="C3 C4 C2" WINDOWS="-1 64" bash tools/cfg_sweep.sh
