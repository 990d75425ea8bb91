#!/bin/bash
# Round-6 GPU sessions (one gpurun call each; every GPU step under its own time limit,
# stopping at the first crash / timeout).
#   bash tools/r06_session.sh tests     GPU tests + smoke
#   bash tools/r06_session.sh inflight  frames-in-flight A/B at N = 1 (tools/inflight_ab.sh)
#   bash tools/r06_session.sh mfma      sustained MFMA rates incl. the scaled form
set -o pipefail
mkdir -p gpurun_out
for step in "$@"; do
  case $step in
    tests)
      echo "=== pytest"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/pytest_gpu.txt 2>&1
      rc=$?; tail -15 gpurun_out/pytest_gpu.txt
      [ $rc -eq 0 ] || exit $rc
      echo "=== smoke"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 \
        || { tail -20 gpurun_out/smoke.txt; exit 1; }
      tail -1 gpurun_out/smoke.txt ;;
    inflight)
      bash tools/inflight_ab.sh || exit 1 ;;
    sdma)
      timeout -k 10 120 python tools/sdma_probe.py --out gpurun_out/sdma_probe_r06.jsonl > gpurun_out/sdma.txt 2>&1 \
        || { tail gpurun_out/sdma.txt; exit 1; } ;;
    inflight2)  # the reference-shaped configs (README / integration grid), F = 1 / 2 at 20 steps
      SCS="readme integ-n6 integ-n8 integ-n12 integ-n16 integ-n12-s25" FLS="1 2" STEPSLIST=20 \
        OUT=gpurun_out/inflight2_r06.jsonl bash tools/inflight_ab.sh || exit 1 ;;
    mfma)
      timeout -k 10 200 ./build/mfma_rate > gpurun_out/mfma_r06.txt 2>&1 || exit 1
      cat gpurun_out/mfma_r06.txt ;;
    abpk)  # packed-key search: lazy drops (default build) vs the drop branch (build/alt_pkbranch.so)
      cp libbicos_amd/libbicos_amd.so build/cur.so
      for k in 1 2; do for l in cur alt_pkbranch; do
        cp build/$l.so libbicos_amd/libbicos_amd.so
        timeout -k 10 300 python tools/random_search_bench.py --words 1,2 --inputs random_u32,random_u64 \
          --reps 5 > gpurun_out/abpk_rand.txt 2>&1 || { tail gpurun_out/abpk_rand.txt; cp build/cur.so libbicos_amd/libbicos_amd.so; exit 1; }
        python - $l $k >> gpurun_out/abpk_r06.jsonl <<'PY'
import json, sys
for line in open("gpurun_out/abpk_rand.txt"):
    if line.startswith("{"):
        d = json.loads(line); d["build"], d["round"] = sys.argv[1], int(sys.argv[2]); print(json.dumps(d))
PY
        for c in cfg1 integ-n6 integ-n8; do
          timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-host-path \
            --kernel-reps 5 2> gpurun_out/abpk.err | python tools/jl.py gpurun_out/abpk_r06.jsonl build=$l round=$k \
            || { tail gpurun_out/abpk.err; cp build/cur.so libbicos_amd/libbicos_amd.so; exit 1; }
        done
      done; done
      cp build/cur.so libbicos_amd/libbicos_amd.so ;;
    abhost)  # host path: maps band by band on their own stream (default) vs one download (BICOS_HOST_DL=once)
      for k in 1 2; do for dl in band once; do
        BICOS_HOST_DL=$dl timeout -k 10 300 python tools/host_bench.py --reps 9 > gpurun_out/abhost_${dl}_$k.txt 2>&1 || exit 1
        grep '^{' gpurun_out/abhost_${dl}_$k.txt | head -2 | sed "s/^{/{\"dl\": \"$dl\", \"round\": $k, /" >> gpurun_out/abhost_r06.jsonl
      done; done
      BICOS_HOST_TRACE=1 timeout -k 10 300 python tools/host_bench.py --reps 2 > gpurun_out/host_trace_r06.txt 2>&1 || exit 1 ;;
    abhost2)  # host path: one / two upload streams x one download / band-wise downloads
      for k in 1 2; do for v in base up2 band up2band; do
        case $v in base) e="";; up2) e="BICOS_HOST_UPLOAD_STREAMS=2";; band) e="BICOS_HOST_DL=band";;
                   up2band) e="BICOS_HOST_UPLOAD_STREAMS=2 BICOS_HOST_DL=band";; esac
        env $e timeout -k 10 300 python tools/host_bench.py --reps 9 > gpurun_out/abhost_${v}_$k.txt 2>&1 || exit 1
        grep '^{' gpurun_out/abhost_${v}_$k.txt | head -2 | sed "s/^{/{\"variant\": \"$v\", \"round\": $k, /" >> gpurun_out/abhost2_r06.jsonl
      done; done
      BICOS_HOST_UPLOAD_STREAMS=2 BICOS_HOST_TRACE=1 timeout -k 10 300 python tools/host_bench.py --reps 2 > gpurun_out/host_trace_r06_up2.txt 2>&1 || exit 1 ;;
    abcons2)  # the dense-row criterion (ascending col1) on cfg4 and the random / planted searches
      for k in 1 2; do for v in on nodense; do
        case $v in on) e="";; nodense) e="BICOS_DENSE_ROWS=0";; esac
        env $e timeout -k 10 200 python bench.py --config cfg4 --steps 40 --warmup 3 --no-cpu-baseline --no-host-path \
          --kernel-reps 10 2> gpurun_out/abcons.err | python tools/jl.py gpurun_out/abcons2_r06.jsonl variant=$v round=$k \
          || { tail gpurun_out/abcons.err; exit 1; }
        env $e timeout -k 10 300 python tools/random_search_bench.py --words 4 --inputs planted_stereo_n33,random_u128 \
          --reps 5 > gpurun_out/abcons2_rand_${v}_$k.txt 2>&1 || exit 1
      done; done ;;
    pk128)  # packed keys for 128-bit descriptors (variant 68, now with lazy drops) vs the default
      for c in cfg2 cfg5 readme; do
        timeout -k 10 300 python tools/search_sweep.py --config $c --rounds 5 --reps 5 --variants 0:0:0,68:0:0 \
          > gpurun_out/pk128_$c.txt 2>&1 || { tail gpurun_out/pk128_$c.txt; exit 1; }
      done
      timeout -k 10 300 python tools/search_sweep.py --config cfg2 --random --rounds 5 --reps 5 --variants 0:0:0,68:0:0 \
        > gpurun_out/pk128_cfg2_random.txt 2>&1 || { tail gpurun_out/pk128_cfg2_random.txt; exit 1; } ;;
    abpk128)  # the headline shapes: packed-key search + fused agree (default) vs the one-product
              # search + fused agree (BICOS_PK128=0), interleaved twice, N = 1 lines and band 0 of 8
      for k in 1 2; do for v in pk mx; do
        case $v in pk) e="";; mx) e="BICOS_PK128=0";; esac
        for c in cfg2 cfg5 cfg3 readme; do
          env $e timeout -k 10 200 python bench.py --config $c --steps 40 --warmup 3 --no-cpu-baseline --no-host-path \
            --kernel-reps 10 2> gpurun_out/abpk128.err | python tools/jl.py gpurun_out/abpk128_r06.jsonl variant=$v round=$k \
            || { tail gpurun_out/abpk128.err; exit 1; }
        done
        env $e timeout -k 10 200 python bench.py --config cfg2 --band-of 8 --steps 200 --warmup 5 --no-cpu-baseline --no-host-path \
          --kernel-reps 10 2> gpurun_out/abpk128.err | python tools/jl.py gpurun_out/abpk128_r06.jsonl variant=$v round=$k band_of=8 \
          || { tail gpurun_out/abpk128.err; exit 1; }
      done; done ;;
    abcons)  # cfg4: Consistency check in the agree / dense-row reverse search, each switched off
      for k in 1 2; do for v in on nocons nodense off; do
        case $v in on) e="";; nocons) e="BICOS_FUSE_CONS=0";; nodense) e="BICOS_DENSE_ROWS=0";; off) e="BICOS_FUSE_CONS=0 BICOS_DENSE_ROWS=0";; esac
        env $e timeout -k 10 200 python bench.py --config cfg4 --steps 40 --warmup 3 --no-cpu-baseline --no-host-path \
          --kernel-reps 10 2> gpurun_out/abcons.err | python tools/jl.py gpurun_out/abcons_r06.jsonl variant=$v round=$k \
          || { tail gpurun_out/abcons.err; exit 1; }
      done; done
      for v in on nodense; do
        case $v in on) e="";; nodense) e="BICOS_DENSE_ROWS=0";; esac
        env $e timeout -k 10 300 python tools/random_search_bench.py --words 4 --inputs planted_stereo_n33,random_u128 \
          --reps 5 > gpurun_out/abcons_rand_$v.txt 2>&1 || exit 1
      done ;;
    rootload)  # rank 0's gather ingress rehearsed on one GPU: band 0 of an N-way
               # split, 6 frames in flight, alone / + RCCL-shaped receive (16 copy workgroups) /
               # + copy-engine ingress (hipMemcpyDeviceToDeviceNoCU on 1, 2, 4 streams); every mode
               # lands every step's bytes, with the gather pipeline's back pressure; interleaved twice
      for k in 1 2; do for cb in ${RLSETS:-cfg2:8 cfg2:4 cfg2:2 cfg5:8}; do
        c=${cb%%:*}; nb=${cb##*:}
        for m in none proxy16 dma1 dma2 dma4; do
          case $m in
            none) extra= ;;
            proxy16) extra="--root-load proxy --root-load-wgs 16" ;;
            dma*) extra="--root-load dma --root-load-streams ${m#dma}" ;;
          esac
          timeout -k 10 200 python bench.py --config $c --band-of $nb --inflight 6 --steps 400 --warmup 10 \
            --no-cpu-baseline --no-host-path --kernel-reps 0 $extra 2> gpurun_out/rl.err \
            | python tools/jl.py gpurun_out/root_gather_r06.jsonl band_of=$nb root_load=$m pass=$k \
            || { tail gpurun_out/rl.err; exit 1; }
        done
      done; done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
