# One gpurun call = a sequence of named steps, each under its own time limit, stopping at the first failure.
# usage (on the box): bash tools/gpu_steps.sh <tag> <step> [<step> ...]
# steps:
#   tests            every GPU test                      tests=<file or -k expr>  a subset (file path or -k expression)
#   smoke            __graft_entry__.smoke()
#   bench            bench.py default line               bench:<extra bench.py args, comma-separated> (K5:
#                    bench:--camera-shard,--steps,10,--cpu-iters,0  K4: bench:--backbone,efficientnet_b3,--cpu-iters,0)
#   prof             rocprofv3 kernel trace + stats of the default bench (20 steps)
#   encab:<v,v,...>  tools/encoder_ab.py variants        train  the AMP BEVNet training step line
#   encprof:<v>      kernel trace of tools/encoder_ab.py <v> (1 round, 5 iterations)
#   encpmc:<v>:<c,c> one --pmc pass over tools/encoder_ab.py <v> (1 iteration, one stream group)
#   trainprof        kernel trace of 3 AMP training steps
#   pmc:<counters>[:<bench args>]  one rocprofv3 --pmc pass over a 3-step bench (both comma-separated)
#   py:<script,args> any python tool under tools/ (args comma-separated)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
for step in "$@"; do
  name=${step%%[:=]*}; arg=""
  case "$step" in *[:=]*) arg=${step#*[:=]};; esac
  echo "== $step $(date +%T)"
  case "$name" in
    tests)
      if [ -z "$arg" ]; then sel=(tests -m gpu)
      elif [ -e "$arg" ]; then sel=("$arg" -m gpu)
      else sel=(tests -m gpu -k "$arg"); fi
      timeout -k 10 1000 python -u -m pytest "${sel[@]}" -x -q -p no:cacheprovider --timeout 300 \
        --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
      tail -2 $O/smoke.log ;;
    bench) b=bench${arg:+_${arg//[^A-Za-z0-9]/_}}
      timeout -k 10 600 python -u bench.py ${arg//,/ } > $O/$b.log 2>&1; rc=$?; tail -1 $O/$b.log ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
        python3 bench.py --steps 20 --warmup 3 --cpu-iters 0 > $O/prof.log 2>&1; rc=$? ;;
    bprof) d=$O/bprof${arg:+_${arg//[^A-Za-z0-9]/_}}  # kernel trace of a bench variant: bprof:<bench args>
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
        python3 bench.py --steps 10 --warmup 2 --cpu-iters 0 ${arg//,/ } > $O/bprof.log 2>&1; rc=$? ;;
    encab) timeout -k 10 600 python -u tools/encoder_ab.py ${arg//,/ } > $O/encab.log 2>&1; rc=$?
      grep median $O/encab.log; grep MISMATCH $O/encab.log ;;
    encprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/encprof_$arg -o run -- \
        python3 tools/encoder_ab.py $arg --rounds 1 --iters 5 > $O/encprof_$arg.log 2>&1; rc=$? ;;
    encpmc) v=${arg%%:*}; c=${arg#*:}
      timeout -s KILL 120 rocprofv3 --pmc ${c//,/ } --output-format csv -d $O/encpmc_${v}_$(echo $c | md5sum | cut -c1-6) -o run -- \
        python3 tools/encoder_ab.py $v --rounds 1 --iters 1 --stream-groups 1 > $O/encpmc.log 2>&1; rc=$? ;;
    train) timeout -k 10 400 python -u tools/train_step_bench.py --bevnet --amp > $O/train.log 2>&1; rc=$?
      tail -1 $O/train.log ;;
    trainprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tprof -o run -- \
        python3 tools/train_step_bench.py --steps 3 --warmup 1 --bevnet --amp > $O/tprof.log 2>&1; rc=$? ;;
    pmc) c=${arg%%:*}; ba=""; case "$arg" in *:*) ba=${arg#*:};; esac
      d=$O/pmc_${c//,/_}${ba:+_${ba//[^A-Za-z0-9]/_}}
      timeout -s KILL 180 rocprofv3 --pmc ${c//,/ } --output-format csv -d $d -o run -- \
        python3 bench.py --steps 3 --warmup 1 --cpu-iters 0 ${ba//,/ } > $O/pmc.log 2>&1; rc=$? ;;
    py) set -- ${arg//,/ }; s=$1; shift
      timeout -k 10 600 python -u tools/$s "$@" > $O/$(basename $s .py).log 2>&1; rc=$?
      tail -5 $O/$(basename $s .py).log ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  echo "== $step rc=$rc $(date +%T)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
