#!/bin/bash
# One parameterised GPU-box driver (run through gpurun from the repo root):
#   tools/gpu.sh TAG step [step ...]
# steps (each under its own time limit; the script stops at the first failure):
#   tests[=PATTERN]   pytest -m gpu (optionally -k PATTERN; _or_ = ' or ', _and_ = ' and ') -> gpurun_out/TAG_gpu_tests.log
#   smoke             __graft_entry__.smoke()                          -> TAG_smoke.log
#   bench[:ARGS]      python bench.py ARGS (ARGS comma-separated)      -> TAG_bench[_MODE].log
#   prof[:ARGS]       rocprofv3 --kernel-trace --stats of bench ARGS  -> TAG_prof[_MODE]/
#   pmc:KERNEL[:ARGS] FETCH_SIZE and WRITE_SIZE passes of bench ARGS, summarised for KERNEL into
#                     profiles/pmc_latest.json (tools/pmc_traffic.py)  -> TAG_pmc_KERNEL_{f,w}/
#   sq:KERNEL[:ARGS]  two SQ counter passes (MFMA busy, waits, instruction mix) -> TAG_sq_KERNEL{1,2}/
#   py:SCRIPT[:ARGS]  python SCRIPT ARGS                               -> TAG_py_NAME.log
#   ab:LIB[:ARGS]     python bench.py ARGS with ANR_LIB_PATH=ab/LIB.so (an alternative build of the
#                     same C-ABI, e.g. other -D options; same-box A/B)  -> TAG_ab_LIB[_MODE].log
#   trace[:ARGS]      rocprofv3 --kernel-trace (per-dispatch timestamps, no stats) of bench ARGS
#                     (tools/train_trace_summary.py, tools/sdf_batch_trace.py read it) -> TAG_trace[_MODE]/
#   probe[:ARGS]      tools/gemm_probe ARGS (layer-GEMM kernels timed alone; make probe) -> TAG_probe.log
#   probeprof[:ARGS]  the same under rocprofv3 --kernel-trace --stats        -> TAG_probeprof/
#   probecnt:KERNEL:C1+C2[:ARGS]  one --pmc pass over the probe, KERNEL's dispatches -> TAG_pcnt_KERNEL/
#   counters:KERNEL:C1+C2+..[:ARGS]  one --pmc pass with the given counters (<= the per-block limits)
#                     over one bench step                              -> TAG_cnt_KERNEL/
#   env:VAR=VALUE     export VAR for the steps after it; bench / prof / trace logs get _VAR-VALUE
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=$1
shift
mkdir -p gpurun_out
SFX=""
args_of() { echo "$1" | tr ',' ' '; }
# log-name suffix: _MODE, then the other flags (steps / warmup left out), e.g. _train_precision-fp32
mode_of() {
  local m rest t=""
  m=$(echo "$1" | sed -n 's/.*--mode,\([a-z-]*\).*/\1/p')
  rest=$(echo "$1" | sed 's/--mode,[a-z-]*//; s/--steps,[0-9]*//; s/--warmup,[0-9]*//; s/--//g; s/[^a-zA-Z0-9.]\{1,\}/-/g; s/^-//; s/-$//')
  [ -n "$m" ] && t="_$m"
  [ -n "$rest" ] && t="${t}_$rest"
  echo "$t"
}
for step in "$@"; do
  kind=${step%%:*}
  rest=${step#*:}
  [ "$rest" = "$step" ] && rest=""
  case $kind in
    tests|tests=*)
      pat=${step#tests=}
      [ "$pat" = "$step" ] && pat=""
      pat=${pat//_or_/ or }
      pat=${pat//_and_/ and }
      sel=()
      [ -n "$pat" ] && sel=(-k "$pat")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread "${sel[@]}" \
        > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { rc=$?; tail -40 gpurun_out/${TAG}_gpu_tests.log; exit $rc; }
      tail -1 gpurun_out/${TAG}_gpu_tests.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
        || { rc=$?; tail -20 gpurun_out/${TAG}_smoke.log; exit $rc; }
      tail -2 gpurun_out/${TAG}_smoke.log ;;
    bench)
      log=gpurun_out/${TAG}_bench$(mode_of "$rest")$SFX.log
      timeout -k 10 600 python bench.py $(args_of "$rest") > $log 2>&1 || { rc=$?; tail -20 $log; exit $rc; }
      tail -n 1 $log | cut -c1-600 ;;
    prof)
      m=$(mode_of "$rest")$SFX
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof$m -o run --output-format csv -- \
        python bench.py --no-cpu --no-torch-baseline $(args_of "$rest") > gpurun_out/${TAG}_prof$m.log 2>&1 \
        || { rc=$?; tail -20 gpurun_out/${TAG}_prof$m.log; exit $rc; }
      echo "PROF_OK $m" ;;
    pmc)
      k=${rest%%:*}
      a=${rest#*:}
      [ "$a" = "$rest" ] && a=""
      B="python bench.py --steps 1 --warmup 0 --no-cpu --no-exact --no-torch-baseline --no-host-render $(args_of "$a")"
      timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$k" -d gpurun_out/${TAG}_pmc_${k}_f -o f \
        --output-format csv -- $B > gpurun_out/${TAG}_pmc_${k}_f.log 2>&1 || { rc=$?; tail -20 gpurun_out/${TAG}_pmc_${k}_f.log; exit $rc; }
      timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$k" -d gpurun_out/${TAG}_pmc_${k}_w -o w \
        --output-format csv -- $B > gpurun_out/${TAG}_pmc_${k}_w.log 2>&1 || { rc=$?; tail -20 gpurun_out/${TAG}_pmc_${k}_w.log; exit $rc; }
      f=$(ls gpurun_out/${TAG}_pmc_${k}_f/*counter_collection.csv | head -1)
      w=$(ls gpurun_out/${TAG}_pmc_${k}_w/*counter_collection.csv | head -1)
      python tools/pmc_traffic.py "$f" "$w" "$k" "profiles/pmc_${TAG} ($k)" || exit 1 ;;
    sq)
      k=${rest%%:*}
      a=${rest#*:}
      [ "$a" = "$rest" ] && a=""
      B="python bench.py --steps 1 --warmup 0 --no-cpu --no-exact --no-torch-baseline --no-host-render $(args_of "$a")"
      timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$k" \
        -d gpurun_out/${TAG}_sq_${k}1 -o p --output-format csv -- $B > gpurun_out/${TAG}_sq_${k}1.log 2>&1 || exit 1
      timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM \
        SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA --kernel-include-regex "$k" \
        -d gpurun_out/${TAG}_sq_${k}2 -o p --output-format csv -- $B > gpurun_out/${TAG}_sq_${k}2.log 2>&1 || exit 1
      echo "SQ_OK $k" ;;
    py)
      s=${rest%%:*}
      a=${rest#*:}
      [ "$a" = "$rest" ] && a=""
      n=$(basename "$s" .py)
      timeout -k 10 600 python "$s" $(args_of "$a") > gpurun_out/${TAG}_py_$n.log 2>&1 || { rc=$?; tail -30 gpurun_out/${TAG}_py_$n.log; exit $rc; }
      tail -n 3 gpurun_out/${TAG}_py_$n.log | cut -c1-600 ;;
    ab)
      lib=${rest%%:*}
      a=${rest#*:}
      [ "$a" = "$rest" ] && a=""
      [ -f ab/$lib.so ] || { echo "ab/$lib.so missing"; exit 2; }
      log=gpurun_out/${TAG}_ab_${lib}$(mode_of "$a").log
      ANR_LIB_PATH=$PWD/ab/$lib.so timeout -k 10 600 python bench.py $(args_of "$a") > $log 2>&1 || { rc=$?; tail -20 $log; exit $rc; }
      tail -n 1 $log | cut -c1-400 ;;
    trace)
      m=$(mode_of "$rest")$SFX
      timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_trace$m -o run --output-format csv -- \
        python bench.py --no-cpu --no-torch-baseline $(args_of "$rest") > gpurun_out/${TAG}_trace$m.log 2>&1 \
        || { rc=$?; tail -20 gpurun_out/${TAG}_trace$m.log; exit $rc; }
      echo "TRACE_OK $m" ;;
    probe)
      [ -x tools/gemm_probe ] || { echo "tools/gemm_probe missing (make probe)"; exit 2; }
      timeout -k 10 300 tools/gemm_probe $(args_of "$rest") > gpurun_out/${TAG}_probe.log 2>&1 \
        || { rc=$?; tail -20 gpurun_out/${TAG}_probe.log; exit $rc; }
      echo "PROBE_OK" ;;
    probeprof)
      [ -x tools/gemm_probe ] || { echo "tools/gemm_probe missing (make probe)"; exit 2; }
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_probeprof -o run --output-format csv -- \
        tools/gemm_probe $(args_of "$rest") > gpurun_out/${TAG}_probeprof.log 2>&1 \
        || { rc=$?; tail -20 gpurun_out/${TAG}_probeprof.log; exit $rc; }
      echo "PROBEPROF_OK" ;;
    probecnt)
      k=${rest%%:*}
      r2=${rest#*:}
      cs=${r2%%:*}
      a=${r2#*:}
      [ "$a" = "$r2" ] && a=""
      timeout -s KILL 180 rocprofv3 --pmc ${cs//+/ } --kernel-include-regex "$k" -d gpurun_out/${TAG}_pcnt_$k -o p \
        --output-format csv -- tools/gemm_probe $(args_of "$a") > gpurun_out/${TAG}_pcnt_$k.log 2>&1 \
        || { rc=$?; tail -20 gpurun_out/${TAG}_pcnt_$k.log; exit $rc; }
      echo "PROBECNT_OK $k" ;;
    counters)
      k=${rest%%:*}
      r2=${rest#*:}
      cs=${r2%%:*}
      a=${r2#*:}
      [ "$a" = "$r2" ] && a=""
      B="python bench.py --steps 1 --warmup 0 --no-cpu --no-exact --no-torch-baseline --no-host-render $(args_of "$a")"
      timeout -s KILL 180 rocprofv3 --pmc ${cs//+/ } --kernel-include-regex "$k" -d gpurun_out/${TAG}_cnt_$k -o p \
        --output-format csv -- $B > gpurun_out/${TAG}_cnt_$k.log 2>&1 || { rc=$?; tail -20 gpurun_out/${TAG}_cnt_$k.log; exit $rc; }
      echo "COUNTERS_OK $k" ;;
    env)
      export "$rest"
      v=${rest//=/-}
      v=${v##*/}  # a path value: its file name
      SFX="${SFX}_${v}"
      echo "ENV $rest" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo ALL_OK
