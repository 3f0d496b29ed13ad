# decisive-fixture probe at config 3 with 4 stories; then the default bench + round profile
mkdir -p gpurun_out/r3m
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u tools/decisive_probe.py 4 tl200 tl50_q50 tl50_q50_kl50 tl20_q200 tl50 > gpurun_out/r3m/probe.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3m/bench.log 2>&1 || exit 1
bash tools/profile_round.sh r3m
