#!/bin/bash
# One gpurun session: each GPU step has its own time limit; stop at the first
# crash/timeout (exit >= 2 other than pytest's 1 = test failures).
set -u
mkdir -p gpurun_out
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name: $*" | tee -a gpurun_out/session.log
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.txt" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
    tail -3 "gpurun_out/$name.txt" | tee -a gpurun_out/session.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)" | tee -a gpurun_out/session.log; exit $rc; fi
    return 0
}
for step in "$@"; do
    case $step in
        valu) run valu 120 ./build/valu_peak ;;
        mfma) run mfma 200 ./build/mfma_rate ;;
        sweepband)  # geometry candidates for narrow row bands (N=8: 192 rows, N=4: 384)
            run sweepband192 300 python tools/search_sweep.py --rows 192 --variants ${SV192:-0:0:0,64:4:8:0,64:2:8:0,64:4:4:32,64:2:4:32,64:4:8:48}
            run sweepband384 300 python tools/search_sweep.py --rows 384 --variants ${SV384:-0:0:0,64:4:8:0,64:2:8:0,64:4:4:32,64:4:8:48} ;;
        bands) run bands 300 python tools/band_bench.py --config ${SC:-cfg2} ;;
        hostov) run hostov 300 python tools/host_overhead.py ;;
        planeread) run planeread 120 ./build/plane_read ;;
        dep) run dep 200 ./build/dep_bench ;;
        smoke) run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
        pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
        pytestk) run pytest_gpu 900 python -m pytest tests -m gpu -q ;;
        bench) run bench 600 python bench.py --steps 20 --warmup 3 ;;
        benchf) run benchf 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path ;;
        bench3) run bench3 600 python bench.py --config cfg3 --steps 10 --warmup 2 --no-cpu-baseline --no-host-path ;;
        ab1|ab3|ab2|ab4)  # A/B on one box: current lib vs build/alt.so (same bench, interleaved twice)
            c=cfg${step#ab}
            cp libbicos_amd/libbicos_amd.so build/cur.so
            for k in 1 2; do
                cp build/cur.so libbicos_amd/libbicos_amd.so
                run ${step}_cur$k 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline
                cp build/alt.so libbicos_amd/libbicos_amd.so
                run ${step}_alt$k 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline
            done
            cp build/cur.so libbicos_amd/libbicos_amd.so ;;
        subpix) run subpix 300 python tools/subpix_bench.py ;;
        subpixs) run subpixs 300 python tools/subpix_bench.py --ns 16,33 --steps 0.5,0.2,0.1,0.05 ;;
        host) run host 400 python tools/host_bench.py ;;
        host2) run host2 400 python tools/host_bench.py --reps 9 ;;
        hosttrace) BICOS_HOST_TRACE=1 run hosttrace 400 python tools/host_bench.py --reps 2 ;;
        hostknobs)
            for th in ${HOST_THREADS:-4 8 16}; do
                BICOS_HOST_THREADS=$th run hostk_${th} 300 python tools/host_bench.py --reps 7
            done ;;
        pytestsub) run pytest_sub 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "subpix or cfg3 or match_bit_exact" ;;
        absearch)  # search kernel alone: current lib vs build/alt.so, interleaved twice
            cp libbicos_amd/libbicos_amd.so build/cur.so
            for k in 1 2; do
                cp build/cur.so libbicos_amd/libbicos_amd.so
                run absearch_cur${k}_${SC:-cfg2} 300 python tools/search_sweep.py --config ${SC:-cfg2} --variants 0:0:0
                cp build/alt.so libbicos_amd/libbicos_amd.so
                run absearch_alt${k}_${SC:-cfg2} 300 python tools/search_sweep.py --config ${SC:-cfg2} --variants 0:0:0
            done
            cp build/cur.so libbicos_amd/libbicos_amd.so ;;
        abn)  # search kernel alone over several builds (LIBS="alt share2 ..." = build/<x>.so), interleaved twice
            cp libbicos_amd/libbicos_amd.so build/cur.so
            for k in 1 2; do
                for l in ${LIBS}; do
                    cp build/$l.so libbicos_amd/libbicos_amd.so
                    run abn_${l}_${k}_${SC:-cfg2} 300 python tools/search_sweep.py --config ${SC:-cfg2} --variants 0:0:0
                done
            done
            cp build/cur.so libbicos_amd/libbicos_amd.so ;;
        abag)  # agree/subpixel stages alone: current lib vs build/alt.so, interleaved twice
            cp libbicos_amd/libbicos_amd.so build/cur.so
            for k in 1 2; do
                cp build/cur.so libbicos_amd/libbicos_amd.so
                run abag_cur$k 300 python tools/subpix_bench.py --ns ${AGNS:-33,40,16} --rows 1536
                cp build/alt.so libbicos_amd/libbicos_amd.so
                run abag_alt$k 300 python tools/subpix_bench.py --ns ${AGNS:-33,40,16} --rows 1536
            done
            cp build/cur.so libbicos_amd/libbicos_amd.so ;;
        subpix16) run subpix16 300 python tools/subpix_bench.py --depth 2 --ns 8,16,24,33 ;;
        bench4) run bench4 600 python bench.py --config cfg4 --steps 10 --warmup 2 --no-cpu-baseline --no-host-path ;;
        stagekib)
            for c in cfg5 cfg4f; do for k in 0 40 32; do
                BICOS_SEARCH_STAGE_KIB=$k run stage_${c}_$k 300 python bench.py --config $c --steps 8 --warmup 2 --no-cpu-baseline --no-host-path
            done; done ;;
        bench5) run bench5 600 python bench.py --config cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-host-path ;;
        sweepv) run sweepv_${SC:-cfg2}_${SROWS:-all} 600 python tools/search_sweep.py --config ${SC:-cfg2} ${SROWS:+--rows $SROWS} --variants $SV ;;
        pmcmx) run pmcmx 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/pmcmx -o run --output-format csv -- python tools/search_sweep.py --rounds 1 --reps 2 --variants ${SV:-64:8:8} ;;
        pmcclk) for c in ${CLKCFG:-cfg2 cfg4}; do
                run pmcclk_$c 120 timeout -s KILL 100 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU -d gpurun_out/pmcclk_$c -o run --output-format csv -- python tools/search_sweep.py --config $c --rounds 1 --reps 3 --variants ${SV:-0:0:0}
            done ;;
        diag)  # search-kernel floors: diagnostic builds (tools/build_diag.sh) vs the real one
            cp libbicos_amd/libbicos_amd.so build/cur.so
            run diag_real_${SC:-cfg2} 300 python tools/search_sweep.py --config ${SC:-cfg2} --variants ${SV:-0:0:0}
            for d in ${DIAGS:-1 2 3}; do
                cp build/diag$d.so libbicos_amd/libbicos_amd.so
                run diag${d}_${SC:-cfg2} 300 python tools/search_sweep.py --config ${SC:-cfg2} --variants ${SV:-0:0:0}
            done
            cp build/cur.so libbicos_amd/libbicos_amd.so ;;
        sweep8) run sweep8 600 python tools/search_sweep.py --rows 192 --variants 0:0:0:0,16:2:8:4,16:2:8:8,16:4:8:8 ;;
        sweep48) run sweep48 600 python tools/search_sweep.py --rows 384 --variants 0:0:0:0,16:2:8:2,16:2:8:4,16:2:8:8 && python tools/search_sweep.py --rows 768 --variants 0:0:0:0,16:2:8:1,16:2:8:2,16:2:8:4 && python tools/search_sweep.py --config cfg5 --rows 270 --variants 0:0:0:0,16:2:8:4,16:2:8:8 ;;
        sweep5) run sweep5 600 python tools/search_sweep.py --config cfg5 --rows 270 --variants 0:0:0:0,16:2:8:1,16:2:8:2,16:2:8:4 ;;
        rehearse2) run rehearse2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --steps 5 --warmup 1 --no-cpu-baseline --no-host-path ;;
        pmcsub) run pmcsub 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmcsub -o run --output-format csv -- python bench.py --config cfg3 --steps 2 --warmup 1 --no-cpu-baseline --kernel-reps 1 ;;
        prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path ;;
        pmcf) run pmcf 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --kernel-reps 2 ;;
        pmcw) run pmcw 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --kernel-reps 2 ;;
        pmcs) run pmcs 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/pmcs -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --kernel-reps 2 ;;
        pmcl) run pmcl 600 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_VALU_INT32 TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmcl -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --kernel-reps 2 ;;
        selflaunch2) run selflaunch2 600 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 1 --no-cpu-baseline --no-host-path ;;
        benchcfgs)  # one bench line per BASELINE config at N=1 (cfg2 with the CPU baseline)
            run bench_cfg2 600 python bench.py --config cfg2 --steps 20 --warmup 3
            for c in cfg3 cfg4 cfg5 cfg1; do
                run bench_$c 600 python bench.py --config $c --steps 20 --warmup 3 --no-host-path --cpu-seconds 8
            done ;;
        profcfg)  # rocprofv3 kernel stats of one config (SC=cfgN)
            run prof_${SC:-cfg2} 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${SC:-cfg2} -o run --output-format csv -- python bench.py --config ${SC:-cfg2} --steps 10 --warmup 2 --no-cpu-baseline --no-host-path ;;
        profiso)  # rocprofv3 kernel stats with one frame at a time (no cross-frame kernel overlap), SCS="cfg2 cfg3 ..."
            for c in ${SCS:-cfg2}; do
                run profiso_$c 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profiso_$c -o run --output-format csv -- python bench.py --config $c --steps 10 --warmup 2 --inflight 1 --no-cpu-baseline --no-host-path
            done ;;
        abpipe)  # frame pipeline (N=1 and N=8 bands, 1 and 3 streams): current lib vs build/alt.so, interleaved twice
            cp libbicos_amd/libbicos_amd.so build/cur.so
            for k in 1 2; do
                cp build/cur.so libbicos_amd/libbicos_amd.so
                run abpipe_cur$k 300 python tools/frame_pipe_bench.py --ns 1,8 --streams 1,3 --rounds 2
                cp build/alt.so libbicos_amd/libbicos_amd.so
                run abpipe_alt$k 300 python tools/frame_pipe_bench.py --ns 1,8 --streams 1,3 --rounds 2
            done
            cp build/cur.so libbicos_amd/libbicos_amd.so ;;
        abtf)  # transform stage alone (reference kernel-bench shapes) + one config's frame: current lib vs build/alt.so
            cp libbicos_amd/libbicos_amd.so build/cur.so
            for k in 1 2; do
                for l in cur alt; do
                    cp build/$l.so libbicos_amd/libbicos_amd.so
                    run abtf_${l}$k 300 python tools/ref_kernel_bench.py --stages transform --reps 40
                    run abtfb_${l}$k 300 python bench.py --config ${SC:-readme} --steps 10 --warmup 2 --no-cpu-baseline --no-host-path
                done
            done
            cp build/cur.so libbicos_amd/libbicos_amd.so ;;
        abbench)  # whole bench lines over several builds (LIBS="a b ..." = build/<x>.so, SCS configs), interleaved twice
            cp libbicos_amd/libbicos_amd.so build/cur.so
            for k in 1 2; do
                for c in ${SCS:-cfg2}; do
                    for l in ${LIBS}; do
                        cp build/$l.so libbicos_amd/libbicos_amd.so
                        run abb_${c}_${l}_$k 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-host-path
                    done
                done
            done
            cp build/cur.so libbicos_amd/libbicos_amd.so ;;
        pmchead)  # HBM bytes per in-frame dispatch at HEAD: FETCH_SIZE and WRITE_SIZE passes per
                  # config / band (PMCSETS="cfg2:1 cfg2:8 ..."), summarised by tools/pmc_summary.py
            mkdir -p gpurun_out/pmc
            python -c "import bench; print(bench.kernel_source_hash())" > gpurun_out/pmc/source_sha
            for cb in ${PMCSETS:-cfg2:1 cfg2:2 cfg2:4 cfg2:8 cfg3:1 cfg4:1 cfg5:1 cfg5:8 readme:1 cfg1:1}; do
                c=${cb%%:*}; nb=${cb##*:}
                for set in FETCH_SIZE WRITE_SIZE; do
                    run pmc_${c}_b${nb}_${set} 150 timeout -s KILL 140 rocprofv3 --pmc $set -d gpurun_out/pmc/${c}__b${nb}__${set} -o run --output-format csv -- python bench.py --config $c --band-of $nb --steps 3 --warmup 1 --spinup-ms 0 --kernel-reps 0 --inflight 1 --no-cpu-baseline --no-host-path
                done
            done ;;
        pmcstall)  # stall / occupancy / memory-latency counters of the in-frame kernels (PMCSETS as above)
            mkdir -p gpurun_out/pmc
            python -c "import bench; print(bench.kernel_source_hash())" > gpurun_out/pmc/source_sha
            for cb in ${PMCSETS:-cfg2:1}; do
                c=${cb%%:*}; nb=${cb##*:}
                run pmc_${c}_b${nb}_sq 150 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum -d gpurun_out/pmc/${c}__b${nb}__sq -o run --output-format csv -- python bench.py --config $c --band-of $nb --steps 3 --warmup 1 --spinup-ms 0 --kernel-reps 0 --inflight 1 --no-cpu-baseline --no-host-path
                run pmc_${c}_b${nb}_mem 150 timeout -s KILL 140 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_SPI_STALL_sum GRBM_GUI_ACTIVE SQ_WAVES -d gpurun_out/pmc/${c}__b${nb}__mem -o run --output-format csv -- python bench.py --config $c --band-of $nb --steps 3 --warmup 1 --spinup-ms 0 --kernel-reps 0 --inflight 1 --no-cpu-baseline --no-host-path
            done ;;
        dmag)  # the copy-engine gather rehearsed with gloo ranks sharing the one GPU (IPC-mapped slots, hipMemcpyAsync), 2 and 3 ranks, + the rccl-form rehearsal
            run dmag2 600 python bench.py --gpus 2 --backend gloo --gather dma --steps 5 --warmup 1 --no-cpu-baseline --no-host-path
            run dmag3 600 python bench.py --gpus 3 --backend gloo --gather dma --config cfg3 --steps 5 --warmup 1 --no-cpu-baseline --no-host-path
            run rcclg2 600 python bench.py --gpus 2 --backend gloo --gather rccl --steps 5 --warmup 1 --no-cpu-baseline --no-host-path ;;
        benchg2)  # the N=2 path rehearsed with gloo ranks sharing the one GPU (all line fields)
            run benchg2 600 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 1 --cpu-seconds 4 ;;
        tunepipe)  # search geometries that leave wave slots for the other frames' HBM stages
            run tunepipe 600 python tools/frame_pipe_bench.py --ns 1 --streams 1,2,3 --rounds 2 --reps 40 --tunes ${TUNES:-0:0:0:0,64:4:4:48,64:4:4:40,64:4:6:64,64:2:8:64,64:4:8:64} ;;
        refk) run refk 600 python tools/ref_kernel_bench.py --out gpurun_out/ref_kernel_bench.jsonl ;;
        randsearch) run randsearch 600 python tools/random_search_bench.py --out gpurun_out/random_search.jsonl ;;
        rootload)  # rank 0 of an N = 8 run on one GPU: band-of-8 with 3 frames in flight, without / with the gather ingress (CU copy kernel, DMA)
            for k in 1 2; do for c in ${SCS:-cfg2 cfg5}; do
                for m in ${RLMODES:-none proxy8 proxy16 proxy16hp proxy32 dma}; do
                    case $m in
                        none) extra= ;;
                        proxy*hp) w=${m#proxy}; extra="--root-load proxy --root-load-wgs ${w%hp} --root-load-high-priority" ;;
                        proxy*) extra="--root-load proxy --root-load-wgs ${m#proxy}" ;;
                        *) extra="--root-load $m" ;;
                    esac
                    run rl_${c}_${RLN:-8}_${m}$k 300 python bench.py --config $c --band-of ${RLN:-8} --inflight ${INFL:-3} --steps 400 --warmup 10 --no-cpu-baseline --no-host-path --kernel-reps 0 $extra
                done
            done; done ;;
        revprof)  # kernel trace of the random-descriptor searches: kept col1 / full reverse
            run revprof_kept 300 rocprofv3 --kernel-trace --stats -d gpurun_out/revprof_kept -o run --output-format csv -- python tools/random_search_bench.py --words 4 --inputs random_u128 --reps 5
            BICOS_REV_FULL=1 run revprof_full 300 rocprofv3 --kernel-trace --stats -d gpurun_out/revprof_full -o run --output-format csv -- python tools/random_search_bench.py --words 4 --inputs random_u128 --reps 5 ;;
        hostdma) run hostdma 300 python tools/host_dma_probe.py ;;
        fuseab)  # agree fused into the search launch vs separate (BICOS_FUSE_AGREE=0), SCS configs, interleaved REPS times
            for k in $(seq ${REPS:-2}); do
                for c in ${SCS:-cfg2}; do
                    run fuse_${c}_on$k 300 python bench.py --config $c --steps 40 --warmup 3 --no-cpu-baseline --no-host-path ${BARGS:-}
                    BICOS_FUSE_AGREE=0 run fuse_${c}_off$k 300 python bench.py --config $c --steps 40 --warmup 3 --no-cpu-baseline --no-host-path ${BARGS:-}
                done
            done
            run fuseprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fuseprof -o run --output-format csv -- python bench.py --config ${SC:-cfg2} --steps 10 --warmup 2 --inflight 1 --no-cpu-baseline --no-host-path --kernel-reps 0 ;;
        bandfl)  # frames in flight for row bands: band 0 of BANDS-way splits of SCS configs, F = FLS, interleaved twice
            for k in 1 2; do
                for c in ${SCS:-cfg2 cfg5}; do
                    for b in ${BANDS:-8 4}; do
                        for f in ${FLS:-3 4 6}; do
                            run bandfl_${c}_${b}_f${f}_$k 300 python bench.py --config $c --band-of $b --inflight $f --steps 100 --warmup 5 --no-cpu-baseline --no-host-path --kernel-reps 0
                        done
                    done
                done
            done ;;
        swband)  # search geometries for row bands (cfg2 N = 8 / 4 bands and the whole frame), back to back
            for r in ${ROWS:-192 384 1536}; do
                run swband_$r 300 python tools/search_sweep.py --config ${SC:-cfg2} --rows $r --rounds 7 --reps 10 \
                    --variants "${VARS:-0:0:0,64:2:8:0,64:4:8:0,64:2:8:40,64:2:8:48,64:4:8:48,64:2:4:32,64:4:4:32,64:4:4:0}"
            done ;;
        bandprof)  # kernel stats of band 0 of a BAND-way split (default cfg2 / 8), one frame at a time and 3 in flight
            for f in 1 3; do
                run bandprof_${SC:-cfg2}_${BAND:-8}_f$f 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bandprof_${SC:-cfg2}_${BAND:-8}_f$f -o run --output-format csv -- python bench.py --config ${SC:-cfg2} --band-of ${BAND:-8} --steps 100 --warmup 5 --inflight $f --no-cpu-baseline --no-host-path --kernel-reps 0
            done ;;
        revrand)  # random-descriptor searches (32/64/128-bit) with the compacted reverse search vs the full one
            run revrand_kept 600 python tools/random_search_bench.py --words 1,2,4 --out gpurun_out/random_search_kept.jsonl
            BICOS_REV_FULL=1 run revrand_full 600 python tools/random_search_bench.py --words 1,2,4 --out gpurun_out/random_search_full.jsonl
            for k in 1 2; do
                run bench4_kept$k 300 python bench.py --config cfg4 --steps 20 --warmup 3 --no-cpu-baseline --no-host-path
                BICOS_REV_FULL=1 run bench4_full$k 300 python bench.py --config cfg4 --steps 20 --warmup 3 --no-cpu-baseline --no-host-path
            done ;;
        revprof4)  # cfg4 kernel stats one frame at a time: compacted reverse, full reverse
            run revprof4_kept 300 rocprofv3 --kernel-trace --stats -d gpurun_out/revprof4_kept -o run --output-format csv -- python bench.py --config cfg4 --steps 10 --warmup 2 --inflight 1 --no-cpu-baseline --no-host-path --kernel-reps 0
            BICOS_REV_FULL=1 run revprof4_full 300 rocprofv3 --kernel-trace --stats -d gpurun_out/revprof4_full -o run --output-format csv -- python bench.py --config cfg4 --steps 10 --warmup 2 --inflight 1 --no-cpu-baseline --no-host-path --kernel-reps 0 ;;
        revab)  # Consistency's reverse search over the kept col1 vs the full reverse pass (BICOS_REV_FULL=1)
            run randsearch_kept 600 python tools/random_search_bench.py --words 1,2,4 --out gpurun_out/random_search_kept.jsonl
            BICOS_REV_FULL=1 run randsearch_full 600 python tools/random_search_bench.py --words 1,2,4 --out gpurun_out/random_search_full.jsonl
            for k in 1 2; do
                run bench4_kept$k 300 python bench.py --config cfg4 --steps 20 --warmup 3 --no-cpu-baseline --no-host-path
                BICOS_REV_FULL=1 run bench4_full$k 300 python bench.py --config cfg4 --steps 20 --warmup 3 --no-cpu-baseline --no-host-path
            done ;;
        benchall)  # one bench line per BASELINE config + the README shape (cfg2 with host path)
            run bench_cfg2 300 python bench.py --config cfg2 --steps 20 --warmup 3
            for c in cfg3 cfg4 cfg5 readme cfg1; do
                run bench_$c 300 python bench.py --config $c --steps 20 --warmup 3 --no-host-path --cpu-seconds 8
            done ;;
        *) echo "unknown step $step" ;;
    esac
done
