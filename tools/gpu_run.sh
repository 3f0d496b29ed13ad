#!/bin/bash
# One GPU-box run recipe for every experiment (replaces the per-round rNN*.sh one-offs).
# Run on the GPU box from the repo root:
#   bash tools/gpu_run.sh TAG STEP [STEP ...]
# Output goes to gpurun_out/TAG/. Each step has its own time limit. The first failing step ends
# the script, and so does a time limit, an abort or a fault: nothing is retried.
# Steps:
#   tests[:ARGS]     pytest -m gpu over ARGS (default: tests)      -> pytest_gpu.log
#   smoke            __graft_entry__.smoke()                          -> smoke.log
#   bench[:ARGS]     python bench.py ARGS                             -> bench.log (appended)
#   py:SCRIPT ARGS   python SCRIPT ARGS                               -> <script>.log (appended)
#   bin:PROG ARGS    a program built here beforehand (e.g. tools/bw_mix) -> <prog>.log (appended)
#   attn-ab:NAME     rocprof kernel stats of tools/attn_bench.py, ab/libmmseq_NAME.so vs the
#                    tree, alternated twice                           -> attn_{NAME,tree}_stats.csv
#   epi-ab:NAME      tools/gemm_epi_bench.py, NAME vs tree, twice     -> epi_{NAME,tree}.log
#   bench-ab:NAME    short bench (config 3 only), NAME vs tree, twice -> bench_{NAME,tree}.log
#   kstats:SCRIPT ARGS  rocprof kernel stats of python SCRIPT ARGS    -> <script>_stats.csv
#   kstats-env:VAR=VAL:SCRIPT ARGS  the same with VAR=VAL exported   -> <script>_VAR<VAL>_stats.csv
#   env-ab:VAR[:SCRIPT ARGS]  the short config-3 bench (or python SCRIPT ARGS) with VAR=0 vs VAR=1,
#                    alternated twice (e.g. env-ab:MMSEQ_ROWS, env-ab:MMSEQ_ROWS:tools/c5_train.py bf16 3)
#                                                                     -> envab_VAR{0,1}.log
#   lib-ab:NAME:SCRIPT ARGS  python SCRIPT ARGS with ab/libmmseq_NAME.so vs the tree, alternated
#                    twice (e.g. lib-ab:base:tools/ln_bench.py bwd)   -> <script>_{NAME,tree}.log
#   pmc:NAME:CTRS:SCRIPT ARGS  one rocprofv3 --pmc pass (CTRS space-free, comma-separated, within
#                    the per-block limits) over python SCRIPT ARGS  -> pmc_NAME.csv
#   profile          tools/profile_round.sh TAG (kernel stats + PMC of the default bench)
#   dp2-gloo         the 2-rank data-parallel path on this one GPU over gloo (4 stories per rank,
#                    the bench line with its all-reduce diagnostics) -> bench_dp2_gloo.log
set -euo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
tag=${1:?tag}; shift
out=gpurun_out/$tag
mkdir -p "$out"
short="--no-cpu-baseline --no-config2 --no-config5 --no-rn50 --no-gemm-timer"

with_lib() {  # with_lib NAME|tree -> sets MMSEQ_BENCH_LIB for the A/B variant
  if [ "$1" = tree ]; then unset MMSEQ_BENCH_LIB; else export MMSEQ_BENCH_LIB=ab/libmmseq_$1.so; fi
}

kstats() {  # kstats DEST_CSV python-args...
  local dest=$1; shift
  local d="$out/kt_$$"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o kt -- \
    python3 "$@" >> "${dest%.csv}.log" 2>&1
  cat "$(find "$d" -name 'kt_kernel_stats.csv' | head -n1)" >> "$dest"
  rm -rf "$d"
}

for step in "$@"; do
  name=${step%%:*}; arg=""
  [ "$name" != "$step" ] && arg=${step#*:}
  echo "== $step" >&2
  case $name in
    tests)
      # eval: ARGS may quote a -k expression, e.g. 'tests:-k "a or b" tests/test_x.py'
      eval timeout -k 10 900 python -u -m pytest -q -rs --maxfail 20 --timeout 300 --timeout-method thread \
        "${arg:-tests}" -m gpu > "$out/pytest_gpu.log" 2>&1 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 ;;
    bench)
      timeout -k 10 600 python -u bench.py $arg >> "$out/bench.log" 2>&1 ;;
    py)
      s=$(basename "${arg%% *}" .py)
      timeout -k 10 600 python -u $arg >> "$out/$s.log" 2>&1 ;;
    bin)
      s=$(basename "${arg%% *}")
      timeout -k 10 300 $arg >> "$out/$s.log" 2>&1 ;;
    attn-ab|epi-ab|bench-ab)
      for v in "$arg" tree "$arg" tree; do
        with_lib "$v"
        case $name in
          attn-ab) kstats "$out/attn_${v}_stats.csv" tools/attn_bench.py 1; timeout -k 10 200 python3 tools/attn_bench.py 1 >> "$out/attn_${v}.log" 2>&1 ;;
          epi-ab) timeout -k 10 200 python3 tools/gemm_epi_bench.py 4 >> "$out/epi_$v.log" 2>&1 ;;
          bench-ab) timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 $short --fwd-steps 0 \
                      >> "$out/bench_$v.log" 2>&1 ;;
        esac
      done
      unset MMSEQ_BENCH_LIB ;;
    kstats)
      s=$(basename "${arg%% *}" .py)
      kstats "$out/${s}_stats.csv" $arg ;;
    kstats-env)
      kv=${arg%%:*}; cmd=${arg#*:}
      s=$(basename "${cmd%% *}" .py)
      export "${kv?}"
      kstats "$out/${s}_${kv%%=*}${kv#*=}_stats.csv" $cmd
      unset "${kv%%=*}" ;;
    env-ab)
      var=${arg%%:*}; cmd=""
      [ "$var" != "$arg" ] && cmd=${arg#*:}
      for v in 0 1 0 1; do
        if [ -n "$cmd" ]; then
          env "$var=$v" timeout -k 10 300 python3 $cmd >> "$out/envab_$var$v.log" 2>&1
        else
          env "$var=$v" timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 $short --fwd-steps 0 \
            >> "$out/envab_$var$v.log" 2>&1
        fi
      done ;;
    lib-ab)
      lname=${arg%%:*}; cmd=${arg#*:}
      s=$(basename "${cmd%% *}" .py)
      for v in "$lname" tree "$lname" tree; do
        with_lib "$v"
        timeout -k 10 300 python3 $cmd >> "$out/${s}_$v.log" 2>&1
      done
      unset MMSEQ_BENCH_LIB ;;
    pmc)
      pn=${arg%%:*}; rest=${arg#*:}; ctrs=${rest%%:*}; cmd=${rest#*:}
      d="$out/pmc_$$"
      timeout -s KILL 120 rocprofv3 --pmc ${ctrs//,/ } --output-format csv -d "$d" -o pm -- \
        python3 $cmd >> "$out/pmc_$pn.log" 2>&1
      cat "$(find "$d" -name 'pm_counter_collection.csv' | head -n1)" > "$out/pmc_$pn.csv"
      rm -rf "$d" ;;
    profile)
      bash tools/profile_round.sh "$tag" ;;
    dp2-gloo)
      timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --dist-backend gloo \
        --batch 4 --micro 4 --steps 3 --warmup 1 $short --fwd-steps 0 > "$out/bench_dp2_gloo.log" 2>&1 ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo "gpu_run $tag done" >&2
