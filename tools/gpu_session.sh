#!/usr/bin/env bash
# One GPU-box session: named steps, each under its own time limit; the session
# stops at the first fault, abort, segfault or timeout (exit >= 2 other than
# pytest's "tests failed" = 1).  Logs go to gpurun_out/<step>.log.
# Usage: tools/gpu_session.sh [steps...]   (default: smoke tests bench prof)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${*:-smoke tests bench prof}

run() {  # name limit cmd...
    local name=$1 lim=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name exit=$rc"
    tail -n 4 "gpurun_out/$name.log" | cut -c1-1500
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name exit $rc"; exit $rc; fi
    if [ $rc -eq 1 ] && [ "$name" != "tests" ]; then echo "STOP: $name failed"; exit 1; fi
    return 0
}

for s in $STEPS; do
    case $s in
        smoke) run smoke 300 python __graft_entry__.py smoke ;;
        tests) run tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
        testk) # the GPU tests whose names match PYTEST_K
               run testk 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
                   -p no:cacheprovider -k "${PYTEST_K:?}" ;;
        bench) run bench 600 python bench.py ;;
        quick) run bench_quick 300 python bench.py --no-cpu --steps 10 ;;
        frames) for f in 4 9 36; do run bench_f$f 300 python bench.py --no-cpu --no-dropin --steps 20 --frames $f || exit 1; done ;;
        split) RT_RESOLVE=split run bench_split 300 python bench.py --no-cpu --steps 10 ;;
        shard8) run bench_shard8 300 python bench.py --no-cpu --no-dropin --steps 10 --shard-of 8 ;;
        shards) for n in 2 4 8; do run bench_shard$n 300 python bench.py --no-cpu --no-dropin --steps 10 --shard-of $n || exit 1; done ;;
        rccl)  run rccl 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rccl -o rccl \
                   -- python tools/rccl_group_probe.py ;;
        fixup) run fixup 900 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_parity.py -x -v --timeout 300 \
                   --timeout-method thread -p no:cacheprovider \
                   -k "headline or consecutive or side_deinterleave or c4 or overflow or redo or packed or rccl or sharded or concurrent or edge or ties or stratified" ;;
        c5)    run c5 900 python -u -m pytest tests/test_gpu_headline.py -x -v --timeout 600 --timeout-method thread \
                   -p no:cacheprovider -k "c5 or c3_shape" ;;
        rcclt) run rcclt 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
                   -p no:cacheprovider -k "rccl_group" ;;
        fetchcal) run fetchcal 300 rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/fcal \
                   -o fcal -- ./tools/fetch_probe && \
               run fetchcalw 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/fcal \
                   -o wcal -- ./tools/fetch_probe && \
               python tools/fetch_calib.py gpurun_out/fcal/fcal_counter_collection.csv gpurun_out/fetch_calib.json \
                   gpurun_out/fcal/wcal_counter_collection.csv ;;
        rehearse) RT_BENCH_REHEARSE=1 run rehearse2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                      --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu ;;
        spp4)  run bench_spp4 300 python bench.py --no-cpu --steps 5 --spp 4 ;;
        ptests) run ptests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -x -v --timeout 600 \
                   --timeout-method thread -p no:cacheprovider -k "paths or c5 or spp_one" ;;
        paths0) RT_PATHS_PRIMARY=0 run bench_paths0 300 python bench.py --paths --no-cpu --steps 3 --warmup 1 ;;
        paths) run bench_paths 300 python bench.py --paths --steps 3 --warmup 1 ;;
        prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
                   -- python bench.py --steps 30 --warmup 4 --no-cpu --no-dropin ;;
        pmc)   run pmc 900 rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/pmc -o fetch \
                   -- python bench.py --steps 1 --warmup 0 --frames 36 --no-cpu --no-dropin --key-out gpurun_out/pmc_key.txt && \
               run pmcw 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o write \
                   -- python bench.py --steps 1 --warmup 0 --frames 36 --no-cpu --no-dropin && \
               RT_RESOLVE=split run pmcs 900 rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_sum --output-format csv \
                   -d gpurun_out/pmc -o walkonly -- python bench.py --steps 1 --warmup 0 --frames 36 --no-cpu --no-dropin && \
               python tools/pmc_traffic.py gpurun_out/pmc/fetch_counter_collection.csv \
                   gpurun_out/pmc/write_counter_collection.csv gpurun_out/pmc_key.txt gpurun_out/pmc_traffic.json \
                   k_trace_packet gpurun_out/pmc/walkonly_counter_collection.csv ;;
        pmcpaths) run pmcp 900 rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/pmcp -o fetch \
                   -- python bench.py --paths --steps 1 --warmup 0 --no-cpu --key-out gpurun_out/pmcp_key.txt && \
               run pmcpw 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcp -o write \
                   -- python bench.py --paths --steps 1 --warmup 0 --no-cpu && \
               python tools/pmc_traffic.py gpurun_out/pmcp/fetch_counter_collection.csv \
                   gpurun_out/pmcp/write_counter_collection.csv gpurun_out/pmcp_key.txt gpurun_out/pmc_traffic_paths.json \
                   ${PATHS_KERNEL:-queue} ;;
        profpaths) run profp 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profp -o paths \
                   -- python bench.py --paths --steps 3 --warmup 1 --no-cpu ;;
        variants) for v in raytracingdemo_amd/variants/librtmi355x_*.so; do
                      n=$(basename "$v" .so); RT_LIB=$PWD/$v run "bench_${n#librtmi355x_}" 300 \
                          python bench.py --no-cpu --no-dropin --steps 10 || exit 1; done ;;
        pvariants) run bench_paths_base 300 python bench.py --paths --no-cpu --steps 3 --warmup 1 || exit 1
                   for v in raytracingdemo_amd/variants/librtmi355x_*.so; do
                      n=$(basename "$v" .so); RT_LIB=$PWD/$v run "bench_paths_${n#librtmi355x_}" 300 \
                          python bench.py --paths --no-cpu --steps 3 --warmup 1 || exit 1; done ;;
        vab)   # A/B, interleaved: the shipped library and every variant, VAB_REPS rounds, 20 steps each
               for rep in $(seq 1 ${VAB_REPS:-2}); do
                   for v in "" raytracingdemo_amd/variants/librtmi355x_*.so; do
                       n=$(basename "${v:-librtmi355x_base}" .so); n=${n#librtmi355x_}
                       RT_LIB=${v:+$PWD/$v} run "vab${VAB_TAG:-}_${n}_$rep" 300 python bench.py --no-cpu --no-dropin --steps ${AB_STEPS:-20} \
                           --shard-of ${AB_SHARD:-1} || exit 1
                       python -c "import json; l=[x for x in open('gpurun_out/vab${VAB_TAG:-}_${n}_$rep.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']; print('RESULT', '${VAB_TAG:-}', '$n', $rep, d['value'], d['ms_per_step'], r['kernel_ms_avg'], r['kernel_ms_span_avg'])" || true
                   done
               done ;;
        pab)   # config c5 A/B, interleaved: the shipped library and every variant, VAB_REPS rounds
               for rep in $(seq 1 ${VAB_REPS:-2}); do
                   for v in "" raytracingdemo_amd/variants/librtmi355x_*.so; do
                       n=$(basename "${v:-librtmi355x_base}" .so); n=${n#librtmi355x_}
                       RT_LIB=${v:+$PWD/$v} run "pab${VAB_TAG:-}_${n}_$rep" 300 python bench.py --paths --no-cpu --steps 3 \
                           --warmup 1 || exit 1
                       python -c "import json; l=[x for x in open('gpurun_out/pab${VAB_TAG:-}_${n}_$rep.log') if x.startswith('{')][-1]; d=json.loads(l); print('RESULT paths', '$n', $rep, d['value'], d['ms_per_step'])" || true
                   done
               done ;;
        stall) # stall hunt: STALL_RUNS entries "label|env|args" (env/args may be empty), STALL_REPS rounds
               IFS=';' read -ra cfgs <<< "${STALL_RUNS:?}"
               for rep in $(seq 1 ${STALL_REPS:-3}); do
                   for c in "${cfgs[@]}"; do
                       IFS='|' read -r lab envs args <<< "$c"
                       env $envs timeout -k 10 300 python bench.py --no-cpu --no-dropin --steps ${AB_STEPS:-20} $args \
                           > gpurun_out/stall_${lab}_$rep.log 2>&1
                       rc=$?; echo "stall_${lab}_$rep exit=$rc"; [ $rc -ne 0 ] && { tail -n 5 gpurun_out/stall_${lab}_$rep.log; exit $rc; }
                       python -c "import json; l=[x for x in open('gpurun_out/stall_${lab}_$rep.log') if x.startswith('{')][-1]; d=json.loads(l); print('RESULT', '$lab', $rep, d['value'], d['ms_per_step'], d['settle_steps'])" || true
                   done
               done ;;
        phases) # dynamic per-phase instruction counts (tools/phase_counts.py): shipped, split walk, and the
               # phase-doubled measurement builds variants/librtmi355x_dblnode.so / _dblleaf.so
               PMC="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE"
               for cfg in base split dblnode dblleaf; do
                   case $cfg in
                       base) e="X=1" ;; split) e="RT_RESOLVE=split" ;;
                       *) e="RT_LIB=$PWD/raytracingdemo_amd/variants/librtmi355x_$cfg.so" ;;
                   esac
                   env $e timeout -k 10 600 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/ph_$cfg -o p \
                       -- python bench.py --steps 1 --warmup 0 --frames 36 --no-cpu --no-dropin > gpurun_out/ph_$cfg.log 2>&1
                   rc=$?; echo "ph_$cfg exit=$rc"; [ $rc -ne 0 ] && { tail -n 5 gpurun_out/ph_$cfg.log; exit $rc; }
               done
               python tools/phase_counts.py gpurun_out/phase_counts.txt base=gpurun_out/ph_base/p_counter_collection.csv \
                   split=gpurun_out/ph_split/p_counter_collection.csv dblnode=gpurun_out/ph_dblnode/p_counter_collection.csv \
                   dblleaf=gpurun_out/ph_dblleaf/p_counter_collection.csv --stats=gpurun_out/ph_base.log ;;
        pwrite) # c5 WRITE_SIZE per kernel (one counted + 2 timed poses) for the shipped library and every variant
               for v in "" raytracingdemo_amd/variants/librtmi355x_*.so; do
                   n=$(basename "${v:-librtmi355x_base}" .so); n=${n#librtmi355x_}
                   RT_LIB=${v:+$PWD/$v} run "pw_$n" 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pw_$n \
                       -o w -- python bench.py --paths --steps 1 --warmup 0 --no-cpu || exit 1
                   python tools/pmc_kernels.py gpurun_out/pw_$n/w_counter_collection.csv --per 2 > gpurun_out/pw_$n.txt || true
               done ;;
        cold)  # first-launch cost in fresh processes: the shipped library and every variant (tools/cold_launch.py)
               for v in "" raytracingdemo_amd/variants/librtmi355x_*.so; do
                   n=$(basename "${v:-librtmi355x_base}" .so); n=${n#librtmi355x_}
                   RT_LIB=${v:+$PWD/$v} run "cold_$n" 600 python tools/cold_launch.py --reps ${COLD_REPS:-4} \
                       --out gpurun_out/cold_$n.json || exit 1
               done ;;
        vshards) for v in raytracingdemo_amd/variants/librtmi355x_*.so; do
                      n=$(basename "$v" .so); RT_LIB=$PWD/$v run "bench_${n#librtmi355x_}_s8" 300 \
                          python bench.py --no-cpu --no-dropin --steps 10 --shard-of 8 || exit 1; done ;;
        sq)    for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
                           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD" \
                           "SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_TC_DATA_READ_REQ SQC_TC_STALL SQ_INST_LEVEL_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
                           "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
                   pn=$((${pn:-0}+1))
                   run sq$pn 900 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/sq -o sq$pn \
                       -- python bench.py --steps 1 --warmup 0 --frames 36 --no-cpu --no-dropin --key-out gpurun_out/pmc_key.txt || exit 1
               done
               python tools/pmc_summary.py gpurun_out/sq/sq*_counter_collection.csv > gpurun_out/sq_summary.txt
               python tools/pmc_valu.py gpurun_out/pmc_key.txt gpurun_out/pmc_valu.json gpurun_out/sq/sq*_counter_collection.csv ;;
        sqpaths) # the SQ passes of `sq` over one pose of config c5 (bench.py --paths, occlusion rays on)
               for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
                           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD" \
                           "SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SCRATCH_READ SQ_INSTS_SCRATCH_WRITE" \
                           "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
                   pn=$((${pn:-0}+1))
                   run sqp$pn 900 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/sqp -o sqp$pn \
                       -- python bench.py --paths --steps 1 --warmup 0 --no-cpu --key-out gpurun_out/pmcp_key.txt || exit 1
               done
               for k in k_q_ k_sh_; do python tools/pmc_summary.py gpurun_out/sqp/sqp*_counter_collection.csv --match $k; done \
                   > gpurun_out/sqp_summary.txt
               python tools/pmc_valu.py --kernel ${PATHS_KERNEL:-queue} gpurun_out/pmcp_key.txt gpurun_out/pmc_valu_paths.json \
                   gpurun_out/sqp/sqp*_counter_collection.csv ;;
        xprobe) # exchange beside the render (tools/exchange_probe.py): all blocks, one block slot free per CU
               run xprobe7 300 python tools/exchange_probe.py --shard-of 8 --steps 200 ${XPROBE_MODES:+--modes $XPROBE_MODES} && \
               RT_PACKET_BLOCKS_PER_CU=6 run xprobe6 300 python tools/exchange_probe.py --shard-of 8 --steps 200 \
                   ${XPROBE_MODES:+--modes $XPROBE_MODES} ;;
        xtrace) # kernel trace of the probe's RCCL mode with one block slot per CU free
               RT_PACKET_BLOCKS_PER_CU=6 run xtrace 300 rocprofv3 --kernel-trace --stats --output-format csv \
                   -d gpurun_out/xtrace -o x -- python tools/exchange_probe.py --shard-of 8 --steps 50 --modes rccl ;;
        ship8) # rank 0's side of an 8-GPU step simulated on one GPU (bench.py RT_BENCH_SHIP_SIM=2), with the
               # side slot (RT_FLAG_SIDE_SLOT, the default with an exchange) and without; then the render alone
               for rep in 1 2; do
               RT_BENCH_SHIP_SIM=2 run ship8_side$rep 300 python bench.py --no-cpu --no-dropin --steps 40 --shard-of 8 && \
               RT_BENCH_SHIP_SIM=2 RT_BENCH_SIDE_SLOT=0 run ship8_full$rep 300 python bench.py --no-cpu --no-dropin \
                   --steps 40 --shard-of 8 || exit 1; done
               run shard8 300 python bench.py --no-cpu --no-dropin --steps 40 --shard-of 8 ;;
        qpdiag) # path-primary phase timing: the shipped kernel, then timing builds QPDIAG_VARIANTS
               run qpd_base 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/qpd_base -o qp \
                   -- python bench.py --paths --steps 2 --warmup 1 --no-cpu || exit 1
               for v in ${QPDIAG_VARIANTS:-qpdiag1 qpdiag2}; do
                   RT_LIB=$PWD/raytracingdemo_amd/variants/librtmi355x_$v.so run qpd_$v 300 rocprofv3 --kernel-trace \
                       --stats --output-format csv -d gpurun_out/qpd_$v -o qp -- python bench.py --paths --steps 2 \
                       --warmup 1 --no-cpu || exit 1; done ;;
        ab)    # A/B over environment settings: AB_ENVS="A=1 B=2;A=3;..." (one bench per entry)
               i=0; IFS=';' read -ra cfgs <<< "${AB_ENVS:-}"
               for c in "${cfgs[@]}"; do i=$((i+1))
                   echo "--- ab$i: $c"
                   env $c timeout -k 10 300 python bench.py --no-cpu --no-dropin --steps ${AB_STEPS:-20} --shard-of ${AB_SHARD:-1} > gpurun_out/ab$i.log 2>&1
                   rc=$?; echo "ab$i exit=$rc"; [ $rc -ne 0 ] && { tail -n 5 gpurun_out/ab$i.log; exit $rc; }
                   python -c "import json; l=[x for x in open('gpurun_out/ab$i.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']; q=r['per_ray']; print('RESULT', '$c', d['value'], r['kernel_ms_avg'], q['wave_nodes_per_tile'], q['wave_leaves_per_tile'], q['wave_tris_per_tile'], q['tri_tests_fp64'])" || true
               done ;;
        sqlite) # SQ passes 1 and 3 of `sq` for the library RT_LIB names: gpurun_out/sq_${SQ_TAG}
               t=${SQ_TAG:-x}
               for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
                           "SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_TC_DATA_READ_REQ SQC_TC_STALL SQ_INST_LEVEL_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
                   pn=$((${pn:-0}+1))
                   run sq_${t}_$pn 600 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/sq_$t -o sq$pn \
                       -- python bench.py --steps 1 --warmup 0 --frames 36 --no-cpu --no-dropin || exit 1
               done
               python tools/pmc_summary.py gpurun_out/sq_$t/sq*_counter_collection.csv > gpurun_out/sq_summary_$t.txt ;;
        pabenv) # paths A/B: PAB_ENVS="A=1;RT_LIB=...;..." (one paths bench per entry)
               i=0; IFS=';' read -ra cfgs <<< "${PAB_ENVS:-}"
               for c in "${cfgs[@]}"; do i=$((i+1))
                   env $c timeout -k 10 300 python bench.py --paths --no-cpu --steps 3 --warmup 1 > gpurun_out/pab$i.log 2>&1
                   rc=$?; echo "pab$i exit=$rc"; [ $rc -ne 0 ] && { tail -n 5 gpurun_out/pab$i.log; exit $rc; }
                   python -c "import json; l=[x for x in open('gpurun_out/pab$i.log') if x.startswith('{')][-1]; d=json.loads(l); print('RESULT', '$c', d['value'], d['kernel_ms_avg'])" || true
               done ;;
        pdiv)  run pdiv 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY \
                   SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pdiv -o paths \
                   -- python bench.py --paths --steps 1 --warmup 0 --no-cpu && \
               run hdiv 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY \
                   SQ_BUSY_CYCLES --output-format csv -d gpurun_out/hdiv -o head \
                   -- python bench.py --steps 1 --warmup 0 --no-cpu --no-dropin ;;
        ovl)   # consecutive steps on two streams (default) vs one (--no-overlap): full size and shard of 8
               i=0
               for o in "" --no-overlap "" --no-overlap; do i=$((i+1))
                   for sh in 1 8; do
                       timeout -k 10 200 python bench.py --no-cpu --no-dropin --steps 40 --shard-of $sh $o \
                           > gpurun_out/ovl${i}_s$sh.log 2>&1
                       rc=$?; [ $rc -ne 0 ] && { tail -n 5 gpurun_out/ovl${i}_s$sh.log; exit $rc; }
                       python -c "import json; l=[x for x in open('gpurun_out/ovl${i}_s$sh.log') if x.startswith('{')][-1]; d=json.loads(l); print('RESULT', 'shard-of $sh', '$o', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['settle_steps'])" || true
                   done
               done ;;
        wvar)  # per variant library (and the shipped one): the headline's WRITE_SIZE per launch, then its bench
               for v in "" raytracingdemo_amd/variants/librtmi355x_*.so; do
                   n=$(basename "${v:-librtmi355x_base}" .so); n=${n#librtmi355x_}
                   RT_LIB=${v:+$PWD/$v} run wv_$n 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/wv_$n -o w \
                       -- python bench.py --steps 1 --warmup 0 --frames 36 --no-cpu --no-dropin || exit 1
                   python -c "import csv,statistics,re; v=[float(r['Counter_Value']) for r in csv.DictReader(open('gpurun_out/wv_$n/w_counter_collection.csv')) if 'k_trace_packet<' in r['Kernel_Name'] and not re.search(r'k_trace_packet<\d+, \d+, \d+, true', r['Kernel_Name'])]; print('WRITE', '$n', len(v), round(statistics.mean(v)*1024/1e9, 4), 'GB/launch')"
                   RT_LIB=${v:+$PWD/$v} run wb_$n 300 python bench.py --no-cpu --no-dropin --steps 20 || exit 1
                   python -c "import json; l=[x for x in open('gpurun_out/wb_$n.log') if x.startswith('{')][-1]; d=json.loads(l); print('BENCH', '$n', d['value'], d['roofline']['kernel_ms_avg'])"
               done ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "=== session done"
