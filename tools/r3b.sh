mkdir -p gpurun_out/r3b
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_order_gpu.py -m gpu > gpurun_out/r3b/order.log 2>&1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3b/yprof -o y -- python3 $GRAFT_REPO_ROOT/tools/yardstick.py > $GRAFT_REPO_ROOT/gpurun_out/r3b/yard.log 2>&1
