#!/bin/bash
# One GPU session on the box (run through gpurun from the repo root):
#   tools/gpu_check.sh TAG [tests] [smoke] [bench] [prof] [ddp]
# tests  the -m gpu suite (per-test timeout, stops at the first failure)
# smoke  __graft_entry__.smoke()
# bench  the default bench.py line (in-step roofline probe + CPU baseline) -> gpurun_out/TAG_bench.json
# bench32  the same at 32 crops per GPU (the multi-GPU per-rank shape, configs[3]) -> gpurun_out/TAG_bench32.json
# prof   rocprofv3 --kernel-trace --stats of bench.py, cut to the timed steps (tools/kstats.py --window)
# ddp    the 2-rank DDP + SyncBN bench path with both ranks on cuda:0 over gloo (a rehearsal, not a scaling number)
# t:EXPR only the -m gpu tests whose names match EXPR (pytest -k)
# rbench the clip_resnet50 bench line (configs[1]) -> gpurun_out/TAG_rbench.json
# rprof  rocprofv3 --kernel-trace --stats of the clip_resnet50 bench, cut to the timed steps
# pstep  the bench command under rocprofv3: kernel trace + 2 PMC passes, per kernel class (tools/pmc_step.py)
# lab:NAME  tools/lab/bin/NAME (LAB_ARGS) -> gpurun_out/TAG_NAME.txt;  plab:NAME  the same under rocprofv3 --kernel-trace --stats
# Every GPU step has its own time limit and the steps are chained: the first failure ends the session.
set -o pipefail
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for what in "$@"; do
  case $what in
    tests)
      timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > $O/${TAG}_tests.log 2>&1 \
        || { tail -60 $O/${TAG}_tests.log; exit 1; }
      tail -1 $O/${TAG}_tests.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 \
        || { tail -30 $O/${TAG}_smoke.log; exit 1; }
      tail -1 $O/${TAG}_smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py > $O/${TAG}_bench.log 2>&1 || { tail -30 $O/${TAG}_bench.log; exit 1; }
      tail -1 $O/${TAG}_bench.log > $O/${TAG}_bench.json; cut -c1-400 $O/${TAG}_bench.json ;;
    bench32)
      # the multi-GPU runs' per-rank shape (configs[3]: 32 crops per GPU) on this one GPU
      timeout -k 10 600 python -u bench.py --crops-per-gpu 32 --steps 30 --warmup 8 --no-cpu-baseline > $O/${TAG}_bench32.log 2>&1 \
        || { tail -30 $O/${TAG}_bench32.log; exit 1; }
      tail -1 $O/${TAG}_bench32.log > $O/${TAG}_bench32.json; cut -c1-400 $O/${TAG}_bench32.json ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o run -- \
        python3 $R/bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-probe > $O/${TAG}_prof.log 2>&1) \
        || { tail -30 $O/${TAG}_prof.log; exit 1; }
      db=$(find $O/${TAG}_prof -name "*.db" | head -1)
      python3 $R/tools/kstats.py "$db" --window --per 20 --top 45 --csv $O/${TAG}_kstats.csv > $O/${TAG}_kstats.txt \
        || { echo "kstats failed"; exit 1; }
      head -25 $O/${TAG}_kstats.txt ;;
    ddp)
      EBC_BENCH_ONE_DEVICE=1 EBC_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 6 --warmup 3 \
        --no-probe > $O/${TAG}_ddp2.log 2>&1 || { tail -40 $O/${TAG}_ddp2.log; exit 1; }
      tail -1 $O/${TAG}_ddp2.log | cut -c1-400 ;;
    t:*)
      timeout -k 10 900 python -u -m pytest -x -v -s --tb=short --timeout 300 --timeout-method thread -m gpu tests -k "${what#t:}" \
        > $O/${TAG}_tsel.log 2>&1 || { tail -60 $O/${TAG}_tsel.log; exit 1; }
      tail -1 $O/${TAG}_tsel.log ;;
    rbench)
      timeout -k 10 600 python -u bench.py --model clip_resnet50 --steps 20 --warmup 5 > $O/${TAG}_rbench.log 2>&1 \
        || { tail -30 $O/${TAG}_rbench.log; exit 1; }
      tail -1 $O/${TAG}_rbench.log > $O/${TAG}_rbench.json; cut -c1-600 $O/${TAG}_rbench.json ;;
    rprof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_rprof -o run -- \
        python3 $R/bench.py --model clip_resnet50 --steps 10 --warmup 5 --no-cpu-baseline --no-probe > $O/${TAG}_rprof.log 2>&1) \
        || { tail -30 $O/${TAG}_rprof.log; exit 1; }
      db=$(find $O/${TAG}_rprof -name "*.db" | head -1)
      python3 $R/tools/kstats.py "$db" --window --per 10 --top 45 --csv $O/${TAG}_rkstats.csv > $O/${TAG}_rkstats.txt \
        || { echo "kstats failed"; exit 1; }
      [ -n "$KCALLS" ] && python3 $R/tools/kstats.py "$db" --window --top 0 --calls "$KCALLS" > $O/${TAG}_rcalls.txt
      rm -rf $O/${TAG}_rprof
      head -40 $O/${TAG}_rkstats.txt ;;
    pstep)
      # the bench command itself under rocprofv3: a kernel-trace pass and two --pmc passes (each its own run, its own
      # limit), cut to the timed steps and mapped to bench.py's kernel classes (tools/pmc_step.py)
      B="$R/bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-trace --classes-out $O/${TAG}_classes.json"
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_ptrace -o run -- \
        python3 $B > $O/${TAG}_ptrace.log 2>&1) || { tail -30 $O/${TAG}_ptrace.log; exit 1; }
      db=$(find $O/${TAG}_ptrace -name "*.db" | head -1)
      python3 $R/tools/kstats.py "$db" --window --per 10 --top 60 > $O/${TAG}_pkstats.txt || { echo "kstats failed"; exit 1; }
      tail -1 $O/${TAG}_ptrace.log | cut -c1-300
      i=0
      for ctrs in "FETCH_SIZE GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES" \
                  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
                  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
        i=$((i+1))
        (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $ctrs -d $O/${TAG}_pmc$i -o run -- \
          python3 $B > $O/${TAG}_pmc$i.log 2>&1) || { tail -30 $O/${TAG}_pmc$i.log; exit 1; }
      done
      python3 $R/tools/pmc_step.py --classes $O/${TAG}_classes.json $O/${TAG}_pmc1 $O/${TAG}_pmc2 $O/${TAG}_pmc3 \
        --json $O/${TAG}_pmc_step.json > $O/${TAG}_pmc_step.txt || { echo "pmc_step failed"; exit 1; }
      rm -rf $O/${TAG}_pmc1 $O/${TAG}_pmc2 $O/${TAG}_pmc3
      head -12 $O/${TAG}_pmc_step.txt | cut -c1-400 ;;
    lab:*)
      # a lab binary (tools/lab/bin/NAME, built here), its stdout -> gpurun_out/TAG_NAME.txt; LAB_ARGS passes arguments
      name=${what#lab:}
      timeout -k 10 400 $R/tools/lab/bin/$name $LAB_ARGS > $O/${TAG}_$name.txt 2>&1 || { tail -30 $O/${TAG}_$name.txt; exit 1; }
      tail -8 $O/${TAG}_$name.txt ;;
    plab:*)
      # the same under rocprofv3 --kernel-trace --stats: per-kernel-name durations -> gpurun_out/TAG_NAME_stats.csv
      name=${what#plab:}
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_${name}_p -o run -- \
        $R/tools/lab/bin/$name $LAB_ARGS > $O/${TAG}_$name.txt 2>&1) || { tail -30 $O/${TAG}_$name.txt; exit 1; }
      st=$(find $O/${TAG}_${name}_p -name "*kernel_stats.csv" | head -1)
      cp "$st" $O/${TAG}_${name}_stats.csv && rm -rf $O/${TAG}_${name}_p
      cut -d, -f1-8 $O/${TAG}_${name}_stats.csv | head -20 ;;
    *) echo "unknown step $what"; exit 2 ;;
  esac
done
echo "gpu_check $TAG done"
