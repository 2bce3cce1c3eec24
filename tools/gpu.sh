#!/bin/bash
# One parametrized GPU-box launcher (replaces the per-experiment gpu_rNN*.sh
# scripts).  Run from the repo root on the box:
#   bash tools/gpu.sh <tag> <step> [<step> ...]
# Steps (each under its own time limit, chained: the first failure ends the call):
#   tests[=REGEX]   pytest -m gpu (optionally -k REGEX), log gpurun_out/<tag>_pytest.log
#   smoke           __graft_entry__.smoke()
#   bench[=ARGS]    python bench.py ARGS (default: the driver's command), gpurun_out/<tag>_bench.json
#   prof=WHAT       rocprofv3 stats + FETCH/WRITE passes (tools/run_profiles.sh WHAT: kkbox fp64 cfg5 kdd12 outbrain)
#   ab=N:ENV_A:ENV_B[:...]  N alternations of env settings (tools/ab.sh; "OCFFM_X=1" = none), gpurun_out/<tag>_ab.txt
#   pe=ARGS         tools/profile_epoch.py ARGS (per-half timeline)
#   py=SCRIPT       python SCRIPT (an experiment script under tools/)
set -e -o pipefail
tag=$1
shift
out=gpurun_out
mkdir -p $out
export TMPDIR=/tmp
for step in "$@"; do
  name=${step%%=*}
  arg=${step#*=}
  [ "$arg" = "$step" ] && arg=""
  echo "== $tag $step  $(date +%T)"
  case $name in
    tests)
      sel=()
      [ -n "$arg" ] && sel=(-k "$arg")
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${sel[@]}" \
        > $out/${tag}_pytest.log 2>&1 || { tail -60 $out/${tag}_pytest.log; exit 1; }
      tail -3 $out/${tag}_pytest.log;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/${tag}_smoke.log 2>&1
      cat $out/${tag}_smoke.log;;
    bench)
      timeout -k 10 900 python bench.py ${arg:---gpus 1 --steps 20 --warmup 5} > $out/${tag}_bench.json 2> $out/${tag}_bench.err \
        || { tail -30 $out/${tag}_bench.err; exit 1; }
      cat $out/${tag}_bench.json;;
    prof)
      bash tools/run_profiles.sh $tag $arg;;
    ab)
      IFS=: read -r -a parts <<< "$arg"
      bash tools/ab.sh "${parts[@]}"
      cp $out/ab.txt $out/${tag}_ab.txt;;
    pe)
      timeout -k 10 600 python tools/profile_epoch.py $arg > $out/${tag}_pe.txt 2>&1
      head -60 $out/${tag}_pe.txt;;
    py)
      timeout -k 10 900 python $arg > $out/${tag}_py.txt 2>&1 || { tail -40 $out/${tag}_py.txt; exit 1; }
      tail -40 $out/${tag}_py.txt;;
    *) echo "unknown step $step"; exit 2;;
  esac
done
