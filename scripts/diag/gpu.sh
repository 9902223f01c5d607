#!/bin/bash
# The one GPU-box driver (run through gpurun from the repo root).  Steps run in order, each
# under its own time limit; the first failure ends the call (set -e, no retries).
#
# Usage: bash scripts/diag/gpu.sh <tag> <step> [<step> ...]      (output: gpurun_out/<tag>/)
#   tests[=<-k expr>]        pytest -m gpu (all files, or `-k expr`), verbose log
#   smoke                    __graft_entry__.smoke()
#   bench[=<args>]           default bench line (+ args; commas -> spaces), bench_<n>.json
#   trace[=<args>]           rocprofv3 kernel trace of a bench run + prof_vs_line check
#   pmc=<counters>[@<args>]  one rocprofv3 --pmc pass (commas -> spaces) over a bench run
#   traffic                  FETCH_SIZE and WRITE_SIZE passes (GEMM kernels) over the bench
#   gemm=<shapes>[@<libs>]   scripts/bench_gemm.py at T = 180992, alternating libraries
#                            (arms: colon list of "ship", VAR=value[+VAR=value], or a
#                            lib/diag/libmmpt_<x>.so name; files named by the arm)
#   gpmc=<counters>@<shapes> one rocprofv3 --pmc pass over bench_gemm (GEMM kernels)
#   attn[=<libs>]            scripts/bench_attn.py alternating libraries the same way
#   env=<VAR=v,...>          export variables for the following steps
#   gclock=<arms>            in-kernel GEMM clock (s_memtime / s_memrealtime, diag build 7),
#                            alternating arms (e.g. ship:MMPT_GEMM_4P=0)
#   scale                    one-GPU scaling preview (per-rank batch 128/64/32) + C2 / C4 lines
set -euo pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
D=multimodal_llm_pretraining_amd/lib/diag
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
nb=0; ng=0; np=0
# an A/B arm: "ship" (the built library), VAR=value (an environment switch; several joined
# by "+"), or a lib/diag/libmmpt_<name>.so variant
lib_env() { case $1 in ship) echo "";; *=*) echo "${1//+/ }";; *) echo "MMPT_LIB=$D/libmmpt_$1.so";; esac; }
last_json() { python3 -c "import sys; print([l for l in open(sys.argv[1]) if l.startswith('{')][-1], end='')" "$1"; }
for step in "$@"; do
  name=${step%%=*}; arg=""; [ "$name" != "$step" ] && arg=${step#*=}
  case $name in
    tests)
      K=(); [ -n "$arg" ] && K=(-k "$arg")
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
          "${K[@]}" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
      tail -1 "$OUT/tests.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
          || { tail -20 "$OUT/smoke.log"; exit 1; }
      tail -1 "$OUT/smoke.log" ;;
    bench)
      nb=$((nb+1))
      timeout -k 10 600 python -u bench.py ${arg//,/ } > "$OUT/bench_$nb.json" 2> "$OUT/bench_$nb.err" \
          || { tail -20 "$OUT/bench_$nb.err"; exit 1; }
      last_json "$OUT/bench_$nb.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; print('bench', d['value'], d['ms_per_step'], (d.get('clock') or {}).get('median_mhz'), (d.get('gemm_yardstick') or {}).get('tflops'), r.get('frac'), r.get('gemm_compute_stream_tflops'))" ;;
    trace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run \
          -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-yardstick ${arg//,/ } \
          > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || { tail -20 "$OUT/trace_bench.err"; exit 1; }
      python3 scripts/diag/prof_vs_line.py "$OUT/trace_bench.json" "$OUT/trace/run_kernel_stats.csv" \
          "$OUT/prof_check.json" > /dev/null
      echo "trace done" ;;
    pmc)
      ctr=${arg%%@*}; ba=""; [ "$ctr" != "$arg" ] && ba=${arg#*@}
      tag=$(echo "$ctr" | tr ',' '_' | cut -c1-40)${MMPT_GEMM_4P:+_4p$MMPT_GEMM_4P}
      timeout -s KILL 300 rocprofv3 --pmc ${ctr//,/ } -f csv -d "$OUT/pmc_$tag" -o run \
          -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe --no-yardstick ${ba//,/ } \
          > "$OUT/pmc_$tag.json" 2> "$OUT/pmc_$tag.err" || { tail -20 "$OUT/pmc_$tag.err"; exit 1; }
      echo "pmc $ctr done" ;;
    traffic)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex gemm -f csv -d "$OUT/$c" -o run \
            -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe --no-yardstick \
            > "$OUT/$c.json" 2> "$OUT/$c.err" || { tail -20 "$OUT/$c.err"; exit 1; }
      done
      echo "traffic done" ;;
    gemm)
      ng=$((ng+1))
      shp=${arg%%@*}; libs=ship; [ "$shp" != "$arg" ] && libs=${arg#*@}
      for r in 1 2; do
        for l in ${libs//:/ }; do
          env $(lib_env "$l") timeout -k 10 300 python -u scripts/bench_gemm.py --tokens 180992 --iters 10 \
              --no-ref --bias --only "$shp" > "$OUT/gemm${ng}_${l}_$r.jsonl" 2> "$OUT/gemm_$l.err" \
              || { tail -20 "$OUT/gemm_$l.err"; exit 1; }
        done
      done
      python3 - "$OUT" $ng ${libs//:/ } <<'PY'
import json, sys
d, ng, libs = sys.argv[1], sys.argv[2], sys.argv[3:]
names = [f"{l}_{r}" for r in (1, 2) for l in libs]
runs = [{x["shape"]: x for x in map(json.loads, open(f"{d}/gemm{ng}_{n}.jsonl"))} for n in names]
print(f"{'shape':18s} " + " ".join(f"{n:>18s}" for n in names) + "  (us, TF/s)")
for k in runs[0]:
    print(f"{k:18s} " + " ".join(f"{r[k]['mmpt_us']:9.1f} {r[k]['mmpt_tflops']:7.1f}" for r in runs))
PY
      ;;
    gpmc)  # gpmc=<counters>@<shapes>: one PMC pass over bench_gemm (GEMM kernels only)
      np=$((np+1))
      ctr=${arg%%@*}; shp=${arg#*@}
      timeout -s KILL 200 rocprofv3 --pmc ${ctr//,/ } --kernel-include-regex gemm -f csv -d "$OUT/gpmc$np" -o run \
          -- python3 scripts/bench_gemm.py --tokens 180992 --iters 3 --no-ref --bias --only "$shp" \
          > "$OUT/gpmc$np.jsonl" 2> "$OUT/gpmc$np.err" || { tail -20 "$OUT/gpmc$np.err"; exit 1; }
      echo "gpmc$np $ctr done" ;;
    attn)
      libs=${arg:-ship}
      for r in 1 2; do
        for l in ${libs//:/ }; do
          env $(lib_env "$l") timeout -k 10 300 python -u scripts/bench_attn.py --iters 20 \
              > "$OUT/attn_${l}_$r.json" 2> "$OUT/attn_$l.err" || { tail -20 "$OUT/attn_$l.err"; exit 1; }
        done
      done
      echo "attn done" ;;
    env)
      for kv in ${arg//,/ }; do export "$kv"; done ;;
    gclock)  # gclock=<arms>: in-kernel GEMM clock (lib/diag/libmmpt_clock.so, MMPT_GEMM_DIAG=7)
      for r in 1 2; do
        for l in ${arg//:/ }; do
          env MMPT_LIB=$D/libmmpt_clock.so $(lib_env "$l") timeout -k 10 300 python -u \
              scripts/diag/gemm_clock.py > "$OUT/gclock_${l}_$r.jsonl" 2> "$OUT/gclock_$l.err" \
              || { tail -20 "$OUT/gclock_$l.err"; exit 1; }
        done
      done
      cat "$OUT"/gclock_*.jsonl ;;
    scale)
      run() {  # <name> <timeout> <bench args...>
        local n=$1 to=$2; shift 2
        MMPT_FORCE_COLLECTIVES=1 timeout -k 10 "$to" python -u bench.py --no-cpu-baseline --no-yardstick "$@" \
            > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -20 "$OUT/$n.err"; exit 1; }
        python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d.get('comm') or {}; print(sys.argv[2], d['value'], d['ms_per_step'], c.get('busy_ms'), c.get('exposed_ms'))" "$OUT/$n.json" "$n"
      }
      for gb in 128 64 32; do
        for mode in ddp zero_2 zero_3; do
          sh=$mode; [ "$mode" = ddp ] && sh=""
          run "vitp1b_gb${gb}_${mode}" 300 --global-batch "$gb" ${sh:+--sharding $sh} --steps 4 --warmup 2
        done
      done
      run c2_pythia1b_zero1_mbs16 600 --model pythia-1b --sharding zero_1 --micro-batch 16 --steps 2 --warmup 1
      run c4_pythia1b_zero3_ac_gb128 400 --model pythia-1b --sharding zero_3 --activation-checkpointing --global-batch 128 --steps 3 --warmup 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "$TAG done"
