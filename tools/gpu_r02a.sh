set -o pipefail
mkdir -p gpurun_out/r02a
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread > gpurun_out/r02a/pytest.log 2>&1
rc=$?
tail -15 gpurun_out/r02a/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02a/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 200 --warmup 20 > gpurun_out/r02a/bench.log 2>&1 || exit $?
tail -c 3000 gpurun_out/r02a/bench.log
cd /tmp && export TMPDIR=/tmp && export PROBE_MAPS=$GRAFT_REPO_ROOT/gpurun_out/r02a/probe_maps.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02a/probe -o probe -- python3 $GRAFT_REPO_ROOT/tools/tab_exit_probe.py > $GRAFT_REPO_ROOT/gpurun_out/r02a/probe.log 2>&1
echo "probe rc=$?"
tail -5 $GRAFT_REPO_ROOT/gpurun_out/r02a/probe.log
