# full GPU suite + smoke on the tree
mkdir -p gpurun_out/r3s
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu --maxfail 20 > gpurun_out/r3s/pytest_gpu.log 2>&1
echo "suite rc $?" >> gpurun_out/r3s/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s/smoke.log 2>&1
echo "smoke rc $?" >> gpurun_out/r3s/smoke.log
