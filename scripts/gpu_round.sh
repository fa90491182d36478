#!/usr/bin/env bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; the script stops after any crash-like exit
# (timeout 124/137, abort 134, segfault 139) and keeps going after plain failures (1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  case $rc in 0|1|2|5) return 0 ;; *) echo "stopping after crash-like exit $rc"; exit $rc ;; esac
}
STEPS=${STEPS:-"tests smoke bench"}
for s in $STEPS; do
  case $s in
    tests) step gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    bench5) step bench5 600 python bench.py --config 5 ;;
    benchkind) step bench_kind 600 python bench.py --cluster kind ;;
    bench6kind) step bench6_kind 600 python bench.py --config 6 --steps 3 --warmup 1 --device on --cluster kind ;;
    bench6on) step bench6_on 600 python bench.py --config 6 --steps 3 --warmup 1 --device on ;;
    c6cpu) step c6cpu 600 python bench.py --config 6 --steps 10 --warmup 2 --alt none ;;   # 10k pods: finer thread-CPU ticks
    bench6off) step bench6_off 600 python bench.py --config 6 --steps 3 --warmup 1 --device off ;;
    benchref) step bench_refqps 600 python bench.py --steps 2 --warmup 0 --reference-qps ;;
    benchhttp) step bench_http 600 python bench.py --transport http --steps 20 --warmup 5 ;;
    benchhttp5) step bench_http5 600 python bench.py --transport http --config 5 --steps 3 --warmup 1 ;;
    benchhttppy) step bench_http_pyapi 600 python bench.py --transport http --apiserver python --client aiohttp --steps 10 --warmup 2 ;;
    profhttp) step prof_http 600 python scripts/profile_bench.py --out gpurun_out/prof_http.txt --transport http --steps 20 --warmup 5 ;;
    profinproc) step prof_inproc 600 python scripts/profile_bench.py --out gpurun_out/prof_inproc.txt --steps 20 --warmup 5 ;;
    pmc) step pmc 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES --kernel-trace --stats --output-format csv -d gpurun_out/pmc -o dev -- python3 scripts/device_bench.py --nodes 4096 --pods 40 --kinds single,gang4 --paths gpu ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    kbprof) step kbprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kbprof -o kb -- python3 scripts/device_batch_bench.py --nodes 4096 --pods 1032 --batch 256 --modes batch ;;
    kbtrace) step kbtrace 300 python scripts/device_batch_bench.py --nodes 4096,16384 --pods 1032 --batch 256 --modes batch --trace ;;
    ab3)   # same-box A/B of the driver's command: this tree vs round 3's (ab_r3/, git worktree of 809b08c,
           # built in place: `git worktree add ab_r3 809b08c && (cd ab_r3 && python -m yoda_scheduler_amd.ops.build)`)
      [ -d ab_r3 ] || { echo "ab3: no ab_r3/ worktree"; exit 1; }
      mkdir -p gpurun_out/ab3
      for k in 1 2; do
        step "ab3/new_$k" 300 python bench.py --gpus 1 --steps 20 --warmup 5 --alt none
        (cd ab_r3 && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --alt none) \
          > "gpurun_out/ab3/r3_$k.log" 2>&1 || { echo "r3 run rc=$?"; exit 1; }
      done ;;
    counters) rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true ;;
    pmc4)  # k_batch PMC on the kept kernel at 256 / 1024 / 4096 nodes, one pass per counter group
      mkdir -p gpurun_out/pmc4
      for n in 256 1024 4096; do
        step "pmc4/p1_$n" 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
          SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY --kernel-trace --stats --output-format csv -d gpurun_out/pmc4/p1_$n -o k \
          -- python3 scripts/device_batch_bench.py --nodes $n --modes batch --busy 0.3 --pods 264 --batch 256
      done
      for n in 256 1024 4096; do
        step "pmc4/p2_$n" 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT \
          SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH --kernel-trace --stats --output-format csv -d gpurun_out/pmc4/p2_$n -o k \
          -- python3 scripts/device_batch_bench.py --nodes $n --modes batch --busy 0.3 --pods 264 --batch 256
      done ;;
    hiptrace6)  # HIP/HSA API census of config 6 (device scorer on): calls per pod, by API
      step hiptrace6 300 rocprofv3 --hip-trace --hsa-trace --stats --output-format csv -d gpurun_out/hiptrace6 -o c6 \
        -- python3 bench.py --config 6 --steps 3 --warmup 1 --alt none
      python scripts/api_census.py gpurun_out/hiptrace6 > gpurun_out/hiptrace6_census.txt 2>&1 || true ;;
    threads6) step threads6 300 env YODA_BENCH_THREADS=1 python bench.py --config 6 --steps 5 --warmup 1 --alt none ;;
    kbab)   # k_batch A/B: this tree's kernel vs abbin/libyoda_hip_base.so (same box, alternated), bench mix
      mkdir -p gpurun_out/kbab
      for k in 1 2; do
        step "kbab/new_$k" 200 python scripts/device_batch_bench.py --nodes 256,1024,4096 --pods 1032 --batch 256 --modes batch --trace --mix bench
        step "kbab/base_$k" 200 env YODA_HIP_LIB=abbin/libyoda_hip_base.so python scripts/device_batch_bench.py --nodes 256,1024,4096 --pods 1032 --batch 256 --modes batch --trace --mix bench
        for v in abbin/libyoda_hip_v*.so; do   # candidate variants built from a patched copy
          [ -f "$v" ] || continue
          t=$(basename "$v" .so); t=${t#libyoda_hip_}
          step "kbab/${t}_$k" 200 env YODA_HIP_LIB="$v" python scripts/device_batch_bench.py --nodes 256,1024,4096 --pods 1032 --batch 256 --modes batch --trace --mix bench
        done
      done ;;
    geo)    # k_batch geometry at 4096 / 16384 nodes: default vs 64 nodes per block on 8 waves, alternated
      mkdir -p gpurun_out/geo
      for k in 1 2; do
        step "geo/default_$k" 200 python scripts/device_batch_bench.py --nodes 4096,16384 --pods 1032 --batch 256 --modes batch --trace --mix bench
        step "geo/npb64w8_$k" 200 env YODA_DEV_NPB=64 YODA_DEV_BWAVES=8 python scripts/device_batch_bench.py --nodes 4096,16384 --pods 1032 --batch 256 --modes batch --trace --mix bench
        step "geo/npb16w4_$k" 200 env YODA_DEV_NPB=16 YODA_DEV_BWAVES=4 python scripts/device_batch_bench.py --nodes 4096 --pods 1032 --batch 256 --modes batch --trace --mix bench
      done ;;
    pairs)  # k_batch two pods in flight (YODA_DEV_PAIRS=1) vs one, alternated; then the parity suite in PAIRS mode
      mkdir -p gpurun_out/pairs
      for k in 1 2; do
        step "pairs/one_$k" 200 env YODA_DEV_PAIRS=0 python scripts/device_batch_bench.py --nodes 256,1024,4096 --pods 1032 --batch 256 --modes batch --trace --mix bench
        step "pairs/two_$k" 200 env YODA_DEV_PAIRS=1 python scripts/device_batch_bench.py --nodes 256,1024,4096 --pods 1032 --batch 256 --modes batch --trace --mix bench
      done ;;
    testspairs) step gpu_tests_pairs 600 env YODA_DEV_PAIRS=1 python -u -m pytest tests/test_gpu_device_scorer.py -x -v --timeout 120 --timeout-method thread ;;
    altinproc)  # the driver's `alt` (in-process apiserver, Python cycle) three times, + a sampled profile
      mkdir -p gpurun_out/alt
      for k in 1 2 3; do step "alt/inproc_$k" 300 python bench.py --transport inproc --alt none --steps 20 --warmup 5; done
      step alt/sample 300 env YODA_PROF_SAMPLE=1 python scripts/profile_bench.py --out gpurun_out/alt/sample.txt \
        --transport inproc --alt none --steps 20 --warmup 5 ;;
    spread)     # config 3 with every pod carrying a hostname spread constraint, next to plain config 3
      mkdir -p gpurun_out/spread
      for k in 1 2; do
        step "spread/c3_$k" 300 python bench.py --config 3 --steps 20 --warmup 5 --alt none
        step "spread/c3spread_$k" 300 python bench.py --config 3 --steps 20 --warmup 5 --mix-spread 1000 --alt none
      done ;;
    realpods)   # config 3 with PVC pods (claim table) and host-port pods (native NodePorts), next to plain config 3
      mkdir -p gpurun_out/realpods
      for k in 1 2; do
        step "realpods/c3_$k" 300 python bench.py --config 3 --steps 20 --warmup 5 --alt none
        step "realpods/c3pvc_$k" 300 python bench.py --config 3 --steps 20 --warmup 5 --mix-volumes 1000 --alt none
        step "realpods/c3hostport_$k" 300 python bench.py --config 3 --steps 20 --warmup 5 --mix-hostports 1000 --alt none
      done ;;
    mixlog) step mixlog 300 env YODA_BENCH_RUNLOG=1 python bench.py --config 3 --mix-anti 10 --steps 5 --warmup 3 --alt none ;;
    scope6) step scope6 300 env YODA_BENCH_THREADS=2 python bench.py --config 6 --steps 5 --warmup 1 --alt none ;;
    nodegpus)   # BASELINE protocol item 5 on config 3: scheduler CPU per attempted pod at 1/2/4/8 GPUs per node
      mkdir -p gpurun_out/nodegpus
      for g in 1 2 4 8; do step "nodegpus/g$g" 300 python bench.py --config 3 --node-gpus $g --steps 10 --warmup 3 --alt none; done ;;
    mixanti)    # 1000-pod burst with 0 / 10 interleaved required-anti-affinity pods, alternated
      mkdir -p gpurun_out/mixanti
      for k in $(seq 1 ${MIXANTI_REPS:-2}); do for m in 0 10; do
        step "mixanti/m${m}_$k" 300 python bench.py --config 3 --mix-anti $m --steps 20 --warmup 5 --alt none
      done; done ;;
    all)   # every BASELINE config (+ 6) on this box, one JSON line each under gpurun_out/all/
      mkdir -p gpurun_out/all
      for spec in "c3|--config 3 --steps 20 --warmup 5" "c1|--config 1 --steps 20 --warmup 2" \
                  "c2|--config 2 --steps 10 --warmup 2" "c4|--config 4 --steps 10 --warmup 2" \
                  "c5|--config 5 --steps 5 --warmup 2" "c6|--config 6 --steps 5 --warmup 1" \
                  "c6off|--config 6 --steps 2 --warmup 1 --device off" \
                  "c3ref|--config 3 --steps 1 --warmup 0 --reference-qps" "c3b|--config 3 --steps 20 --warmup 5" \
                  "c3kind|--config 3 --steps 20 --warmup 5 --cluster kind" "c1kind|--config 1 --steps 20 --warmup 2 --cluster kind" \
                  "c2kind|--config 2 --steps 10 --warmup 2 --cluster kind" "c4kind|--config 4 --steps 10 --warmup 2 --cluster kind" \
                  "c5kind|--config 5 --steps 5 --warmup 2 --cluster kind" "c6kind|--config 6 --steps 5 --warmup 1 --cluster kind" \
                  "c3anti|--config 3 --steps 20 --warmup 5 --mix-anti 10" "c3spread|--config 3 --steps 20 --warmup 5 --mix-spread 1000" \
                  "c3pvc|--config 3 --steps 20 --warmup 5 --mix-volumes 1000" \
                  "c3hostport|--config 3 --steps 20 --warmup 5 --mix-hostports 1000"; do
        step "all/${spec%%|*}" 300 python bench.py --alt none ${spec#*|}
      done
      python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/all/*.log")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["p50_latency_ms"], d["p99_latency_ms"], d.get("e2e_scheduling_p99_ms"),
          d["cpu_us_per_pod"], d.get("apiserver_cpu_us_per_pod"), d["device_cycles"])
PY
      ;;
  esac
done
echo "=== done"
