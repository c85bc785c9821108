#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel stats.
# Every GPU step has its own time limit; a crash / abort / timeout stops the session.
# Usage: bash tools/gpu_session.sh [tag] [steps...]   (steps: test smoke bench prof)
set -u
TAG=${1:-r01}; shift || true
STEPS=${*:-test smoke bench prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case $1 in 0|1) return 1;; *) return 0;; esac; }   # 0 ok, 1 test failures; else stop
python -c "import fedn_amd.build as b; b.build()" > "$OUT/build.log" 2>&1 || { echo "build failed"; exit 2; }
for s in $STEPS; do
  case $s in
    test)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=20 --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1; rc=$?
      echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"; if fatal $rc; then exit $rc; fi ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
      echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python bench.py > "$OUT/bench.log" 2>&1; rc=$?
      echo "bench rc=$rc"; tail -3 "$OUT/bench.log"; [ $rc -eq 0 ] || exit $rc ;;
    rehearsal)
      # the N>1 code path (strong-scaling line + side fields) with 2 ranks on this box's one GPU (gloo)
      FEDN_AMD_BENCH_ONE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --params 20000000 \
        --clients 16 --fedopt-params 20000000 --waves-params 50000000 --waves-clients 32 > "$OUT/rehearsal.log" 2>&1; rc=$?
      echo "rehearsal rc=$rc"; grep -v amdgpu.ids "$OUT/rehearsal.log" | tail -3; [ $rc -eq 0 ] || exit $rc ;;
    selflaunch)
      # bench.py --gpus 2 WITHOUT torchrun (its own rank launcher), both ranks on this box's GPU (gloo)
      FEDN_AMD_BENCH_ONE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 2 --params 20000000 \
        --clients 16 --fedopt-params 20000000 --waves-params 50000000 --waves-clients 32 --cpu-sample 2000000 \
        --host-clients 4 > "$OUT/selflaunch.log" 2>&1; rc=$?
      echo "selflaunch rc=$rc"; grep -v amdgpu.ids "$OUT/selflaunch.log" | tail -3; [ $rc -eq 0 ] || exit $rc ;;
    selflaunch4)
      # the same with 4 ranks on this box's GPU (the N = 4 geometry: 4-way shards, 3 peers per rank)
      FEDN_AMD_BENCH_ONE_GPU=1 timeout -k 10 600 python bench.py --gpus 4 --steps 5 --warmup 2 --params 20000000 \
        --clients 16 --fedopt-params 20000000 --waves-params 50000000 --waves-clients 32 --cpu-sample 2000000 \
        --host-clients 4 > "$OUT/selflaunch4.log" 2>&1; rc=$?
      echo "selflaunch4 rc=$rc"; grep -v amdgpu.ids "$OUT/selflaunch4.log" | tail -2 | cut -c1-400; [ $rc -eq 0 ] || exit $rc ;;
    selflaunch8)
      # bench.py --gpus 8 at DEFAULT sizes, self-launched, all 8 ranks on this box's one GPU
      FEDN_AMD_BENCH_ONE_GPU=1 timeout -k 10 900 python bench.py --gpus 8 > "$OUT/selflaunch8.log" 2>&1; rc=$?
      echo "selflaunch8 rc=$rc"; grep -v amdgpu.ids "$OUT/selflaunch8.log" | tail -2 | cut -c1-600; [ $rc -eq 0 ] || exit $rc ;;
    rccl1)
      # the N>1 path at world size 1 over a real RCCL communicator (all-gathers as collectives, P2P fences)
      FEDN_AMD_BENCH_RCCL_WORLD1=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 1 --steps 5 --warmup 2 --params 100000000 \
        --clients 64 --fedopt-params 50000000 --waves-params 50000000 --waves-clients 32 --cpu-sample 2000000 \
        > "$OUT/rccl1.log" 2>&1; rc=$?
      echo "rccl1 rc=$rc"; grep -v amdgpu.ids "$OUT/rccl1.log" | tail -3; [ $rc -eq 0 ] || exit $rc ;;
    gtest)
      # a subset of the GPU tests: FEDN_AMD_GTEST = pytest -k expression
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
        -k "$FEDN_AMD_GTEST" > "$OUT/gtest.log" 2>&1; rc=$?
      echo "gtest rc=$rc"; tail -5 "$OUT/gtest.log"; [ $rc -eq 0 ] || exit $rc ;;
    small)
      # small-model rounds (configs[0]'s mnist shapes): latency vs numpy, phase breakdown, host profile
      timeout -k 10 600 python tools/bench_small.py > "$OUT/small.log" 2>&1; rc=$?
      echo "small rc=$rc"; grep -v amdgpu.ids "$OUT/small.log" | tail -10; [ $rc -eq 0 ] || exit $rc
      for k in 2 10 64; do
        timeout -k 10 300 python tools/small_breakdown.py --clients $k >> "$OUT/small_breakdown.log" 2>&1; rc=$?
        [ $rc -eq 0 ] || exit $rc
        timeout -k 10 300 python tools/small_breakdown.py --clients $k --kind fedopt >> "$OUT/small_breakdown.log" 2>&1; rc=$?
        [ $rc -eq 0 ] || exit $rc
      done
      grep -v amdgpu.ids "$OUT/small_breakdown.log"
      timeout -k 10 300 python tools/profile_small.py --clients 10 > "$OUT/small_profile.log" 2>&1; rc=$?
      echo "profile rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    floor)
      # configs[0]'s K = 2 round against the GPU round trip's floor and FEDn's own loop overhead
      timeout -k 10 300 python tools/small_floor.py > "$OUT/floor.log" 2>&1; rc=$?
      echo "floor rc=$rc"; grep -v amdgpu.ids "$OUT/floor.log" | head -2 | cut -c1-900; [ $rc -eq 0 ] || exit $rc ;;
    roundblob)
      # a combiner's round end down to the stored global-model blob: FEDn (numpy loop + np.savez_compressed)
      # vs the plug-in (GPU fold + exact writer), blobs compared byte for byte
      timeout -k 10 600 python tools/bench_round_e2e.py > "$OUT/roundblob.log" 2>&1; rc=$?
      echo "roundblob rc=$rc"; grep -v amdgpu.ids "$OUT/roundblob.log" | tail -2 | cut -c1-700; [ $rc -eq 0 ] || exit $rc ;;
    inflate)
      # host npz decode / encode (CPU only): numpy vs the codec's decoder, one stream split over threads
      timeout -k 10 600 python tools/bench_inflate.py > "$OUT/inflate.log" 2>&1; rc=$?
      echo "inflate rc=$rc"; tail -2 "$OUT/inflate.log" | cut -c1-300; [ $rc -eq 0 ] || exit $rc ;;
    fuzzx)
      # the seeded fuzz on fresh seeds, 4x longer (FEDN_AMD_FUZZ_BASE / FEDN_AMD_FUZZ_SCALE override)
      FEDN_AMD_FUZZ_BASE=${FEDN_AMD_FUZZ_BASE:-100000} FEDN_AMD_FUZZ_SCALE=${FEDN_AMD_FUZZ_SCALE:-4} \
        timeout -k 10 1000 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_fuzz_thresholds.py -m gpu -q \
        --timeout 240 --timeout-method thread -p no:cacheprovider > "$OUT/fuzzx.log" 2>&1; rc=$?
      echo "fuzzx rc=$rc"; tail -2 "$OUT/fuzzx.log"; if fatal $rc; then exit $rc; fi ;;
    micro)
      timeout -k 10 600 python tools/microbench.py > "$OUT/micro.log" 2>&1; rc=$?
      echo "micro rc=$rc"; cat "$OUT/micro.log" | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc ;;
    e2e)
      timeout -k 10 600 python tools/bench_e2e.py > "$OUT/e2e.log" 2>&1; rc=$?
      echo "e2e rc=$rc"; grep -v amdgpu.ids "$OUT/e2e.log" | tail -5; [ $rc -eq 0 ] || exit $rc ;;
    fedopt)
      timeout -k 10 900 python tools/bench_fedopt.py > "$OUT/fedopt.log" 2>&1; rc=$?
      echo "fedopt rc=$rc"; grep -v amdgpu.ids "$OUT/fedopt.log" | tail -8; [ $rc -eq 0 ] || exit $rc ;;
    fedopt_ab)
      timeout -k 10 900 python tools/bench_fedopt.py --ab > "$OUT/fedopt_ab.log" 2>&1; rc=$?
      echo "fedopt_ab rc=$rc"; grep -v amdgpu.ids "$OUT/fedopt_ab.log" | tail -20; [ $rc -eq 0 ] || exit $rc ;;
    layout)
      timeout -k 10 600 python tools/layout_probe.py > "$OUT/layout.log" 2>&1; rc=$?
      echo "layout rc=$rc"; grep -v amdgpu.ids "$OUT/layout.log" | tail -14; [ $rc -eq 0 ] || exit $rc ;;
    roundend)
      timeout -k 10 600 python tools/bench_roundend.py > "$OUT/roundend.log" 2>&1; rc=$?
      echo "roundend rc=$rc"; grep -v amdgpu.ids "$OUT/roundend.log" | tail -6; [ $rc -eq 0 ] || exit $rc ;;
    counters)
      timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1; rc=$?
      echo "counters rc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    ingest)
      timeout -k 10 900 python tools/bench_ingest.py > "$OUT/ingest.log" 2>&1; rc=$?
      echo "ingest rc=$rc"; grep -v amdgpu.ids "$OUT/ingest.log" | tail -4; [ $rc -eq 0 ] || exit $rc ;;
    reduce)
      timeout -k 10 600 python tools/bench_reduce.py > "$OUT/reduce.log" 2>&1; rc=$?
      echo "reduce rc=$rc"; grep -v amdgpu.ids "$OUT/reduce.log" | tail -3; [ $rc -eq 0 ] || exit $rc ;;
    upload)
      timeout -k 10 600 python tools/bench_upload.py > "$OUT/upload.log" 2>&1; rc=$?
      echo "upload rc=$rc"; grep -v amdgpu.ids "$OUT/upload.log" | tail -5; [ $rc -eq 0 ] || exit $rc ;;
    upload100mfile)
      # the same with FEDn's file store stand-in (TempModelStorage: chunks to a file, delete = os.remove),
      # 300 and 400 MB/s per client; the delete breakdown (plug-in copies vs the store) is in the lines
      # (store deletes side by side, then inline one after another: FEDN_AMD_DELETE_WORKERS=0)
      for r in 300 400; do
        for dw in 8 0; do
          timeout -k 10 600 python tools/bench_upload.py --params 100000000 --clients 8 --client-MBps $r --store file \
            --delete-workers $dw >> "$OUT/upload100m_file.log" 2>&1; rc=$?
          [ $rc -eq 0 ] || { echo "upload100mfile rc=$rc"; exit $rc; }
        done
      done
      echo "upload100mfile rc=0"; grep '"what"' "$OUT/upload100m_file.log" | cut -c1-600 ;;
    winprobe)
      # FedAdam steady state with the chip's stores confined to a common clock window (probe library)
      timeout -k 10 600 python tools/fedopt_mix_probe.py --burst "" --opt-g "" \
        --win "${FEDN_AMD_WIN:-8192:1200:0,8191:1200:0,8192:1200:2,10000:1400:0,12000:1600:0,14000:2000:0,16384:2400:0,12000:1000:0,12000:2400:0}" \
        > "$OUT/winprobe.log" 2>&1; rc=$?
      echo "winprobe rc=$rc"; cut -c1-1200 "$OUT/winprobe.log" | tail -3; [ $rc -eq 0 ] || exit $rc ;;
    optwin)
      # FedAdam through the product step with / without the chip-wide store window (probe library)
      timeout -k 10 900 python tools/fedopt_window_probe.py ${FEDN_AMD_OPTWIN:+--winprod "$FEDN_AMD_OPTWIN"} \
        ${FEDN_AMD_OPTWINCG:+--wincg "$FEDN_AMD_OPTWINCG"} ${FEDN_AMD_OPTWINK:+--clients "$FEDN_AMD_OPTWINK"} ${FEDN_AMD_OPTWPE:+--wpe "$FEDN_AMD_OPTWPE"} ${FEDN_AMD_OPTCW2:+--wincw2 "$FEDN_AMD_OPTCW2"} > "$OUT/optwin.log" 2>&1; rc=$?
      echo "optwin rc=$rc"; cut -c1-900 "$OUT/optwin.log" | grep -v amdgpu.ids | tail -6; [ $rc -eq 0 ] || exit $rc ;;
    avgwin)
      # FedAvg's fold (64 and 8 x 100 M fp32) with its stores in a chip-wide clock window (probe library)
      timeout -k 10 600 python tools/window_probe.py ${FEDN_AMD_AVGWIN:+--win "$FEDN_AMD_AVGWIN"} ${FEDN_AMD_AVGDT:+--dtype "$FEDN_AMD_AVGDT"} > "$OUT/avgwin.log" 2>&1; rc=$?
      echo "avgwin rc=$rc"; cut -c1-1500 "$OUT/avgwin.log" | grep -v amdgpu.ids | tail -3; [ $rc -eq 0 ] || exit $rc ;;
    wavewin)
      # FedOpt pipeline waves (8 bf16 updates, fp64 model / pg) with their pg stores in the clock window (probe library)
      timeout -k 10 600 python tools/wave_window_probe.py ${FEDN_AMD_WAVEWIN:+--win "$FEDN_AMD_WAVEWIN"} > "$OUT/wavewin.log" 2>&1; rc=$?
      echo "wavewin rc=$rc"; grep -v amdgpu.ids "$OUT/wavewin.log" | tail -4; [ $rc -eq 0 ] || exit $rc ;;
    mixprobe)
      timeout -k 10 600 python tools/fedopt_mix_probe.py > "$OUT/mixprobe.log" 2>&1; rc=$?
      echo "mixprobe rc=$rc"; cut -c1-700 "$OUT/mixprobe.log" | tail -4; [ $rc -eq 0 ] || exit $rc ;;
    upload100m)
      # 8 x 100 M uploads into an in-memory store (delete = drop the bytes): the plug-in's own tail
      for r in 300 400; do
        timeout -k 10 600 python tools/bench_upload.py --params 100000000 --clients 8 --client-MBps $r \
          >> "$OUT/upload100m.log" 2>&1; rc=$?
        [ $rc -eq 0 ] || { echo "upload100m rc=$rc"; exit $rc; }
      done
      echo "upload100m rc=0"; grep '"what"' "$OUT/upload100m.log" | cut -c1-600 ;;
    pmc)
      # HBM traffic per launch for every workload bench.py reports: one rocprofv3 pass per counter
      # (FETCH_SIZE and WRITE_SIZE cannot share a pass), then profiles/pmc_traffic.json
      sha256sum fedn_amd/libfedagg.so | cut -c1-16 > "$OUT/lib_sha.txt"
      i=0
      for args in "--clients 64" "--clients 8 --fedopt-params 0" "--clients 64 --dtype bf16 --fedopt-params 0"; do
        i=$((i+1))
        for c in FETCH_SIZE WRITE_SIZE; do
          cd /tmp && timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/pmc$i/pmc_$c" -o run -- \
            python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --cpu-sample 0 $args --no-side > "$GRAFT_REPO_ROOT/$OUT/pmc${i}_$c.log" 2>&1; rc=$?
          cd "$GRAFT_REPO_ROOT"; echo "pmc$i $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
        done
      done
      echo "pmc: now run  python tools/pmc_traffic.py --session $OUT  in the build container" ;;
    pmcx)
      # PMC traffic of the workloads that need a process of their own (tools/pmc_workloads.py): the
      # fp32-state FedOpt step and configs[4]'s three wave kernels
      sha256sum fedn_amd/libfedagg.so | cut -c1-16 > "$OUT/lib_sha.txt"
      for wl in f32state waves; do
        for c in FETCH_SIZE WRITE_SIZE; do
          cd /tmp && timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/pmcx_$wl/pmc_$c" -o run -- \
            python3 "$GRAFT_REPO_ROOT/tools/pmc_workloads.py" $wl --steps 3 > "$GRAFT_REPO_ROOT/$OUT/pmcx_${wl}_$c.log" 2>&1; rc=$?
          cd "$GRAFT_REPO_ROOT"; echo "pmcx $wl $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
        done
      done
      echo "pmcx: now run  python tools/pmc_traffic.py --x-session $OUT  in the build container" ;;
    pmcrank)
      # HBM traffic of one rank's fold at N = 2, 4, 8 for every fold + all-gather round count bench.py may
      # choose (AG_ROUNDS; bench.py's N > 1 roofline), replayed on this GPU
      sha256sum fedn_amd/libfedagg.so | cut -c1-16 > "$OUT/lib_sha.txt"
      for n in 2 4 8; do
        for R in 1 2 4 8 16; do
          for c in FETCH_SIZE WRITE_SIZE; do
            cd /tmp && timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/pmcrank${n}_r$R/pmc_$c" -o run -- \
              python3 "$GRAFT_REPO_ROOT/tools/pmc_rank_fold.py" --world $n --ag-rounds $R --steps 2 > "$GRAFT_REPO_ROOT/$OUT/pmcrank${n}_r${R}_$c.log" 2>&1; rc=$?
            cd "$GRAFT_REPO_ROOT"; echo "pmcrank$n r$R $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
          done
        done
      done
      echo "pmcrank: now run  python tools/pmc_traffic.py --rank-session $OUT  in the build container" ;;
    pmcprobe)
      PA="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum GRBM_GUI_ACTIVE"
      PB="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum"
      PC="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum"
      for wl in read sum8 sum64 fold64; do
        for ps in A B C; do
          eval "ctrs=\$P$ps"
          cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv \
            -d "$GRAFT_REPO_ROOT/$OUT/pmcprobe/${wl}_$ps" -o run -- python3 "$GRAFT_REPO_ROOT/tools/pmc_probe.py" $wl \
            > "$GRAFT_REPO_ROOT/$OUT/pmcprobe_${wl}_$ps.log" 2>&1; rc=$?
          cd "$GRAFT_REPO_ROOT"; echo "pmcprobe $wl $ps rc=$rc"; [ $rc -eq 0 ] || exit $rc
        done
      done
      python tools/pmc_probe_report.py "$OUT/pmcprobe" ;;
    prof)
      cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- \
        python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --cpu-sample 0 --host-clients 0 > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1; rc=$?
      cd "$GRAFT_REPO_ROOT"; echo "prof rc=$rc"; tail -2 "$OUT/prof.log"; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
