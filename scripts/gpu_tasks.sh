#!/bin/bash
# One launcher for GPU sessions (replaces the per-session gpu_r0*.sh copies):
#
#   bash scripts/gpu_tasks.sh OUT TASK [TASK ...]
#
# runs the named tasks in order, output under gpurun_out/OUT/, each GPU step under its own
# time limit, stopping at the first failure.  Tasks:
#   tests                 every -m gpu test
#   tests:EXPR            the -m gpu tests selected by -k EXPR (',' for ' ')
#   smoke                 __graft_entry__.smoke()
#   bench[:ARGS]          one bench.py line (ARGS with ',' for ' ') -> OUT/bench.jsonl
#   ck_c5                 C5 shard 0/8 advanced 10^5 steps, checkpoint /tmp/ck_c5_100k.npz
#   prof_c5               kernel trace + PMC of the C5 shard resumed from that checkpoint
#   prof_c4 / prof_c3 / prof_c2 / prof_c3s8
#                         kernel trace + PMC of C4 / C3 / C2 / the 8,192-chain C3 shard
#   stamps_c5 / stamps_c4 per-phase clocks (stamps build) at the C5 checkpoint / C4
#   steady                SURVEY 8d's steady state (10^4 + 10^5 steps: --inner 5000
#                         --warmup 2 --steps 20) on every workload -> OUT/steady.jsonl
#   ab:TAG:ARGS:LIB,LIB.. interleaved A/B of ab/lib_<LIB>.so builds (3 rounds) -> OUT/ab_TAG.jsonl
#                         (LIB@VAR=VALUE: with one environment setting)
#   multi                 bench.py under torch.distributed.run, 2 gloo ranks on device 0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1
shift
mkdir -p "$O"
export TMPDIR=/tmp
CK5=/tmp/ck_c5_100k.npz

line() {  # summary of the last JSON line of a bench output file
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pc=d.get('parity_check') or {}; print(sys.argv[2], '%.4g' % d['value'], 'kernel_ms=%.3f' % d['kernel_ms'], 'mean_cut=%.1f' % d['mean_cut'], 'parity=%s/%s' % (pc.get('equal'), pc.get('chains')))" "$1" "$2"
}

prof() {  # prof TAG "cfg args" ["bench args"]
  CFG_ARGS="$2" BENCH_ARGS="${3:-}" timeout -k 10 1000 bash scripts/profile.sh "$1" > "$O/prof_$1.log" 2>&1 \
    || { echo "profile $1 failed"; tail -20 "$O/prof_$1.log"; return 1; }
  tail -40 "$O/prof_$1.log"
}

run_task() {
  local t=$1
  case $t in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
      local rc=$?
      grep -E "passed|failed" $O/pytest_gpu.log | tail -2
      grep -E "FAILED|^E " $O/pytest_gpu.log | head -20
      return $rc ;;
    tests:*)
      local expr=${t#tests:}; expr=${expr//,/ }
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$expr" > $O/pytest_gpu_k.log 2>&1
      local rc=$?
      grep -E "passed|failed" $O/pytest_gpu_k.log | tail -2
      grep -E "FAILED|^E " $O/pytest_gpu_k.log | head -20
      return $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; return 1; }
      tail -2 $O/smoke.log ;;
    bench:*)
      local a=${t#bench:}; a=${a//,/ }
      timeout -k 10 600 python -u bench.py $a > $O/one.json 2> $O/one.err || { echo "bench $a failed"; tail -5 $O/one.err; return 1; }
      tail -1 $O/one.json >> $O/bench.jsonl
      line $O/one.json "$a" ;;
    ck_c5)
      timeout -k 10 300 python -u bench.py --config c5 --shard 0/8 --warmup 0 --steps 100 --check-chains 0 --no-cpu-baseline --save-checkpoint $CK5 > $O/ck_c5.json 2> $O/ck_c5.err || { tail -5 $O/ck_c5.err; return 1; }
      line $O/ck_c5.json ck_c5 ;;
    prof_c5)
      prof c5steady "--config c5 --shard 0/8 --resume $CK5 --check-chains 0" "--steps 5 --warmup 0 --inner 1000 --no-cpu-baseline --config c5 --shard 0/8 --resume $CK5 --check-chains 0" ;;
    prof_c5:*)  # the same with the library ab/lib_<LIB>.so
      local lib=${t#prof_c5:}
      FLIPWALK_LIB=$PWD/ab/lib_$lib.so prof c5steady_$lib "--config c5 --shard 0/8 --resume $CK5 --check-chains 0" "--steps 5 --warmup 0 --inner 1000 --no-cpu-baseline --config c5 --shard 0/8 --resume $CK5 --check-chains 0" ;;
    prof_c5fresh) prof c5fresh "--config c5 --shard 0/8" ;;
    profile:*)  # profile:TAG:BENCH_ARGS (',' for ' '): profile.sh passes of exactly that protocol
      local r=${t#profile:}; local tag=${r%%:*}; local a=${r#*:}; a=${a//,/ }
      BENCH_ARGS="$a --no-cpu-baseline --check-chains 0 --secondary-inner 0" timeout -k 10 1100 bash scripts/profile.sh $tag > "$O/prof_$tag.log" 2>&1 \
        || { echo "profile $tag failed"; tail -20 "$O/prof_$tag.log"; return 1; }
      grep -E "traffic ->|timed=" "$O/prof_$tag.log" ;;
    prof_c4) prof c4 "--config c4" ;;
    prof_c4r) prof c4r "--config c4 --order random" ;;
    prof_frank) prof frank "--config frank" ;;
    prof_c3) prof c3 "" ;;
    prof_c2) prof c2 "--config c2" ;;
    prof_c3s8) prof c3s8 "--config c3 --shard 0/8" ;;
    prof_c3s4) prof c3s4 "--config c3 --shard 0/4" ;;
    prof_c3s2) prof c3s2 "--config c3 --shard 0/2" ;;
    pmc1:*)  # pmc1:TAG:COUNTERS:ARGS:LIB,LIB..  one PMC pass per library (',' for ' ' in
             # COUNTERS and ARGS), means over the timed dispatches -> OUT/pmc1_TAG.jsonl
      local rest=${t#pmc1:}; local tag=${rest%%:*}; rest=${rest#*:}
      local ctrs=${rest%%:*}; rest=${rest#*:}; local args=${rest%%:*}; local libs=${rest#*:}
      ctrs=${ctrs//,/ }; args=${args//,/ }
      local k=$(echo " $args " | sed -n 's/.* --steps \([0-9]*\) .*/\1/p')
      for v in ${libs//,/ }; do
        local lib=${v%%@*} envs=""
        [ "$lib" != "$v" ] && envs=${v#*@}
        rm -rf $O/pmc1_${tag}_$lib
        env $envs FLIPWALK_LIB=$PWD/ab/lib_$lib.so timeout -s KILL 240 rocprofv3 --pmc $ctrs -d $O/pmc1_${tag}_$lib -o run --output-format csv -- python3 bench.py $args --no-cpu-baseline --check-chains 0 > $O/pmc1_${tag}_$lib.log 2>&1 || { echo "pmc $v failed"; tail -5 $O/pmc1_${tag}_$lib.log; return 1; }
        python3 scripts/pmc_one.py $O/pmc1_${tag}_$lib ${k:-1} $v | tee -a $O/pmc1_$tag.jsonl
      done ;;
    stamps:*)  # stamps:CONFIG:CHAINS[:ENV=VAL] (grid kernel phases, 2 warm launches)
      local r=${t#stamps:}; local cfg=${r%%:*}; r=${r#*:}; local nch=${r%%:*}; local ev=""
      [ "$r" != "$nch" ] && ev=${r#*:}
      env $ev timeout -k 10 300 python -u scripts/stamps.py $cfg $nch 2 > $O/stamps_${cfg}_${nch}${ev:+_$ev}.txt 2>&1 || { tail -5 $O/stamps_${cfg}_${nch}${ev:+_$ev}.txt; return 1; }
      grep -v amdgpu.ids $O/stamps_${cfg}_${nch}${ev:+_$ev}.txt ;;
    stamps_c5)
      timeout -k 10 300 python -u scripts/stamps.py c5 8192 1 $CK5 > $O/stamps_c5_100k.txt 2>&1 || { tail -5 $O/stamps_c5_100k.txt; return 1; }
      grep -v amdgpu.ids $O/stamps_c5_100k.txt ;;
    stamps_c4r)
      timeout -k 10 300 python -u scripts/stamps.py c4r 16384 2 > $O/stamps_c4r.txt 2>&1 || { tail -5 $O/stamps_c4r.txt; return 1; }
      grep -v amdgpu.ids $O/stamps_c4r.txt ;;
    stamps_c4)
      timeout -k 10 300 python -u scripts/stamps.py c4 16384 2 > $O/stamps_c4.txt 2>&1 || { tail -5 $O/stamps_c4.txt; return 1; }
      grep -v amdgpu.ids $O/stamps_c4.txt ;;
    steady)
      for a in "--config c3" "--config c2" "--config c4" "--config c5 --shard 0/8" "--config frank" "--config c3 --shard 0/8"; do
        timeout -k 10 300 python -u bench.py $a --inner 5000 --warmup 2 --steps 20 --no-cpu-baseline --check-chains 2 > $O/one.json 2> $O/one.err || { echo "$a failed"; tail -5 $O/one.err; return 1; }
        tail -1 $O/one.json >> $O/steady.jsonl
        line $O/one.json "$a"
      done ;;
    ab:*)
      local rest=${t#ab:}; local tag=${rest%%:*}; rest=${rest#*:}
      local args=${rest%%:*}; local libs=${rest#*:}
      args=${args//,/ }
      for rep in 1 2 3; do
        for v in ${libs//,/ }; do
          # a lib may carry one environment setting: name@VAR=VALUE
          local lib=${v%%@*} envs=""
          [ "$lib" != "$v" ] && envs=${v#*@}
          env $envs FLIPWALK_LIB=$PWD/ab/lib_$lib.so timeout -k 10 300 python -u bench.py $args --no-cpu-baseline > $O/one.json 2> $O/one.err || { echo "$v failed"; tail -5 $O/one.err; return 1; }
          python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pc=d.get('parity_check') or {}; print(json.dumps({'tag': sys.argv[4], 'lib': sys.argv[2], 'rep': int(sys.argv[3]), 'value': d['value'], 'kernel_ms': d['kernel_ms'], 'parity': [pc.get('equal'), pc.get('chains')]}))" $O/one.json $v $rep $tag | tee -a $O/ab_$tag.jsonl
        done
      done ;;
    shards_c5)  # the 8-GPU C5 job emulated shard by shard at the steady-state protocol
      timeout -k 10 900 bash scripts/shards.sh 8 "--config c5 --steps 20 --warmup 5 --check-chains 2" c5 > $O/shards_c5.log 2>&1 || { tail -5 $O/shards_c5.log; return 1; }
      tail -10 $O/shards_c5.log ;;
    shards_c3)  # the 8-GPU C3 job emulated shard by shard on the driver protocol
      timeout -k 10 600 bash scripts/shards.sh 8 "--config c3 --steps 20 --warmup 5 --check-chains 2" c3 > $O/shards_c3.log 2>&1 || { tail -5 $O/shards_c3.log; return 1; }
      tail -10 $O/shards_c3.log ;;
    shards_c3s)  # the 8-GPU C3 job emulated shard by shard at the steady state
      timeout -k 10 900 bash scripts/shards.sh 8 "--config c3 --inner 5000 --steps 20 --warmup 2 --check-chains 2" c3steady > $O/shards_c3steady.log 2>&1 || { tail -5 $O/shards_c3steady.log; return 1; }
      tail -10 $O/shards_c3steady.log ;;
    multi)
      timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --config c3 --chains 8192 --steps 2 --warmup 1 --backend gloo --same-device --no-cpu-baseline --check-chains 4 > $O/multi.json 2> $O/multi.err || { tail -20 $O/multi.err; return 1; }
      tail -1 $O/multi.json ;;
    *) echo "unknown task $t"; return 2 ;;
  esac
}

for t in "$@"; do
  echo "== $t"
  run_task "$t" || { echo "task $t failed: stopping"; exit 1; }
done
