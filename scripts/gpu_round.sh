#!/bin/bash
# GPU-box session, parameterised by STEPS (the one script for every lease; round 5's one-off
# tools/r5_*.sh are folded in as the steps suite / measure / bench5ab / sel):
#   STEPS="smoke pytest bench prof" (default) ... see the case list below.
# Every GPU step has its own time limit; the script stops at the first fault/abort/timeout.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS="${STEPS:-smoke pytest bench prof}"

run() {  # run NAME SECONDS CMD...
    local name=$1 secs=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "rc=$rc"; tail -n 8 "$OUT/$name.log"
    case $rc in
        0|1) return 0 ;;   # pass, or ordinary test/assert failure: the GPU is fine
        *) echo "STOP after $name (rc=$rc)"; exit $rc ;;
    esac
}

for s in $STEPS; do
  case $s in
    suite)  run suite 1200 python -u -m pytest tests/ -x -v -m gpu --timeout 900 --timeout-method thread ;;
    measure)  # bench line, kernel stats (k = 10, 19), SQ / FETCH_SIZE / WRITE_SIZE passes per config
        B="python3 $ROOT/bench.py --no-cpu-baseline"
        SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
        run bench_default 420 python3 bench.py
        (cd /tmp && run prof10 300 rocprofv3 --kernel-trace --stats -d "$OUT/meas/prof10" -o run --output-format csv -- $B --steps 40 --warmup 5) || exit $?
        (cd /tmp && run prof19 300 rocprofv3 --kernel-trace --stats -d "$OUT/meas/prof19" -o run --output-format csv -- $B --steps 20 --warmup 3 --bits-per-key 19) || exit $?
        i=0
        for a in "--steps 3 --warmup 1" "--steps 3 --warmup 1 --bits-per-key 19" "--config 3 --steps 3 --warmup 1" "--config 5 --steps 2 --warmup 1"; do
          i=$((i+1))
          for c in "$SQ" FETCH_SIZE WRITE_SIZE; do
            tag=$(echo "$c" | cut -c1-5)
            (cd /tmp && run pmc_${tag}_$i 240 rocprofv3 --pmc $c -d "$OUT/meas/${tag}_$i" -o run --output-format csv -- $B $a) || exit $?
          done
        done ;;
    benchq19) run bench_k19q 300 python bench.py --no-cpu-baseline --bits-per-key 19 --steps 50 ;;
    prof5ab) (cd /tmp && run prof5ab 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof5ab" -o run -- python3 "$ROOT/bench.py" --config 5 --steps 3 --warmup 1 --no-cpu-baseline --probe-ab) || exit $? ;;
    sel)    run pytest_sel 1200 python -u -m pytest $PYTEST_ARGS -x -v -m gpu --timeout 300 --timeout-method thread ;;
    bench5ab) run bench_cfg5_ab 900 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --probe-ab ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest_gpu 1200 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ;;
    bench)  run bench 600 python bench.py ;;
    benchq)  run bench_quick 300 python bench.py --no-cpu-baseline ;;
    bench19) run bench_k19 300 python bench.py --no-cpu-baseline --bits-per-key 19 --steps 100 ;;
    k19tests) run pytest_k19 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -v -m gpu -k "19 or config2" --timeout 600 --timeout-method thread ;;
    tile1wg) run bench_tile1wg 300 env VBF_TILE_LDS_MIN=98304 VBF_STAGGER=0 python bench.py --no-cpu-baseline --steps 10 ;;
    benchnostagger) run bench_nostagger 300 env VBF_STAGGER=0 python bench.py --no-cpu-baseline ;;
    benchstagger14) run bench_stagger14 300 env VBF_STAGGER=14 python bench.py --no-cpu-baseline ;;
    ablate) run ablate 300 python tools/ablate.py ;;
    ablate19) run ablate19 300 env ABL_M=1900000000 ABL_K=19 python tools/ablate.py 0 1 2 3 5 8 9 ;;
    rdg6)   run rdg6 300 ./tools/rdg6 ;;
    ubhash) run ubench_hash 300 ./tools/ubench hash ;;
    overlap) run overlap 300 ./tools/overlap ;;
    pmcicache) (cd /tmp && run pmcicache 600 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmcicache" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline) || exit $? ;;
    abprev2) run ab_prev2 600 env AB_LIB=velarixdb_amd/libvbf_prev.so tools/ab_lib.sh 3 ;;
    abprev19) run ab_prev19 600 env AB_LIB=velarixdb_amd/libvbf_prev.so tools/ab_lib.sh 3 --bits-per-key 19 ;;
    abprev3) run ab_prev3 600 env AB_LIB=velarixdb_amd/libvbf_prev.so tools/ab_lib.sh 2 --config 3 --steps 5 --warmup 1 ;;
    abprev5) for i in 1 2; do for lib in "" velarixdb_amd/libvbf_prev.so; do run bench_cfg5_prev$i${lib:+_prev} 600 env VBF_LIB=$lib python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline; grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_cfg5_prev$i${lib:+_prev}.log"; done; done ;;
    abprevmulti) for i in 1 2; do for lib in "" velarixdb_amd/libvbf_prev.so; do run bench_multi_prev$i${lib:+_prev} 300 env VBF_LIB=$lib python bench.py --multi --steps 10 --warmup 2; grep -o '"ms_per_step": [0-9.]*\|"phases".*' "$OUT/bench_multi_prev$i${lib:+_prev}.log" | cut -c1-400; done; done ;;
    abpasses) run ab_passes_parity 900 env AB_PARITY=1 AB_ENVS="VBF_K3_PASSES=4" bash tools/env_ab.sh
              run ab_passes10 600 env AB_ENVS="VBF_K3_PASSES=1 VBF_K3_PASSES=2 VBF_K3_PASSES=4 VBF_K3_PASSES=1 VBF_K3_PASSES=2 VBF_K3_PASSES=4" bash tools/env_ab.sh
              run ab_passes19 600 env AB_ENVS="VBF_K3_PASSES=1 VBF_K3_PASSES=2 VBF_K3_PASSES=4 VBF_K3_PASSES=1 VBF_K3_PASSES=2 VBF_K3_PASSES=4" AB_ARGS="--bits-per-key 19" bash tools/env_ab.sh ;;
    abpasses5) for v in 1 4 2 8 1 4; do run bench_cfg5_passes$v 600 env VBF_K3_PASSES=$v python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline; echo "VBF_K3_PASSES=$v"; grep -o '"ms_per_step": [0-9.]*\|"phases": {[^}]*}[^}]*}' "$OUT/bench_cfg5_passes$v.log" | head -2; done ;;
    probe5) run bench_cfg5_probe 600 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline ;;
    probemultitests) run pytest_probe_multi 900 python -u -m pytest tests/test_gpu_probe.py tests/test_gpu_multi.py tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q -m gpu --timeout 300 --timeout-method thread ;;
    probetests) run pytest_probe_sat 900 python -u -m pytest tests/test_gpu_probe.py -x -q -m gpu --timeout 300 --timeout-method thread ;;
    paritytest) run pytest_parity 900 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread ;;
    abk14) for v in 0 1 0 1; do run bench_cfg5_k14_$v 600 env VBF_K1_4=$v python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline; grep -o '"ms_per_step": [0-9.]*\|"phases": {[^}]*}[^}]*}' "$OUT/bench_cfg5_k14_$v.log"; done ;;
    k14tests) run pytest_k14 900 env VBF_K1_4=1 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q -m gpu -k "4294967295 or saturated or config5" --timeout 600 --timeout-method thread ;;
    abk3cfg5) for v in 10 13 3 1 10 13; do run bench_cfg5_k3_$v 600 env VBF_K3=$v python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --neg-keys 1000000; echo "VBF_K3=$v"; grep -o '"phases": {[^}]*}[^}]*}' "$OUT/bench_cfg5_k3_$v.log"; done ;;
    absat5) for v in 0 1 0 1; do run bench_cfg5_sat$v 600 env VBF_SAT=$v python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline; grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_cfg5_sat$v.log"; done ;;
    prof5) (cd /tmp && run prof5 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof5" -o run -- python3 "$ROOT/bench.py" --config 5 --steps 3 --warmup 1 --no-cpu-baseline) || exit $? ;;
    abrotl) run ab_rotl 600 env AB_LIB=velarixdb_amd/libvbf_ab.so tools/ab_lib.sh 3 ;;
    abrotl19) run ab_rotl19 600 env AB_LIB=velarixdb_amd/libvbf_ab.so tools/ab_lib.sh 3 --bits-per-key 19 ;;
    abrotl3) run ab_rotl3 600 env AB_LIB=velarixdb_amd/libvbf_ab.so tools/ab_lib.sh 2 --config 3 --steps 5 --warmup 1 ;;
    abparity) run pytest_ab_parity 900 env VBF_LIB=velarixdb_amd/libvbf_ab.so python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread ;;
    ablatesst) run ablate_sst 300 python tools/ablate_sst.py ;;
    probephases) run probe_phases 300 python tools/probe_phases.py 10 && run probe_phases19 300 python tools/probe_phases.py 19 ;;
    probephases94) run probe_phases9 300 python tools/probe_phases.py 9 && run probe_phases4 300 python tools/probe_phases.py 4 ;;
    probephasesk) run probe_phases14 300 python tools/probe_phases.py 14 && run probe_phases7 300 python tools/probe_phases.py 7 && run probe_phases21 300 python tools/probe_phases.py 21 ;;
    benchatomic) run bench_atomic 300 python bench.py --no-cpu-baseline --strategy 1 --steps 3 ;;
    bench3) run bench_cfg3 600 python bench.py --config 3 --steps 5 --warmup 1 ;;
    bench3q) run bench_cfg3q 600 python bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline ;;
    bench3nolo) run bench_cfg3_nolo 600 env VBF_LEN_ORDER=0 python bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline ;;
    bench3nostage) run bench_cfg3_nostage 600 env VBF_STAGE_KEYS=0 python bench.py --config 3 --steps 5 --warmup 1 --no-cpu-baseline ;;
    bench5) run bench_cfg5 900 python bench.py --config 5 --steps 3 --warmup 1 ;;
    sst)    run bench_sst 600 python bench.py --sst --steps 5 --warmup 1 ;;
    compact) run bench_compact 600 python bench.py --compact --steps 5 --warmup 1 ;;
    multi)  run bench_multi 600 python bench.py --multi --steps 5 --warmup 1 ;;
    profmultigp) (cd /tmp && run profmultigp 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profmultigp" -o run -- python3 "$ROOT/bench.py" --multi --steps 10 --warmup 2) || exit $? ;;
    probetest) run pytest_probe 900 python -u -m pytest tests/test_gpu_probe.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread ;;
    abprobegp) for v in 0 1 0 1; do run probe_phases_gp$v 300 env VBF_PROBE_GP=$v python tools/probe_phases.py; done ;;
    multitest) run pytest_multi 600 python -u -m pytest tests/test_gpu_multi.py -x -v -m gpu --timeout 300 --timeout-method thread ;;
    abmultigp) for v in 0 1 0 1; do run bench_multi_gp$v 300 env VBF_MULTI_GP=$v python bench.py --multi --steps 10 --warmup 2; grep -o '"ms_per_step": [0-9.]*\|"phases".*' "$OUT/bench_multi_gp$v.log"; done ;;
    e2e)    run bench_e2e 600 python bench.py --e2e --steps 5 --warmup 1 ;;
    e2efresh) run bench_e2e_fresh 600 python bench.py --e2e --e2e-fresh-out --steps 5 --warmup 1 ;;
    memtable) run bench_memtable 300 python bench.py --memtable ;;
    fanout) run bench_fanout 600 python bench.py --fanout --steps 3 --warmup 1 ;;
    fanoutab) run bench_fanout_ab 900 bash -c 'for a in "" "--fanout-reuse"; do for h in 1 0; do echo "== H2D_DIRECT=$h $a"; VBF_H2D_DIRECT=$h python bench.py --fanout --steps 3 --warmup 1 $a | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({m: (round(v[\"total_ms\"],1), round(v[\"loop_ms\"],1), round(v[\"materialise_ms\"],1)) for m, v in d[\"modes\"].items()})"; done; done' ;;
    prof19) (cd /tmp && run prof19 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof19" -o run -- python3 "$ROOT/bench.py" --bits-per-key 19 --steps 20 --warmup 3 --no-cpu-baseline) || exit $? ;;
    profmulti) (cd /tmp && run profmulti 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profmulti" -o run -- python3 "$ROOT/bench.py" --multi --steps 10 --warmup 2) || exit $? ;;
    dist2spawn) run bench_dist2_spawn 300 env VBF_SHARE_DEVICE=1 VBF_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline ;;
    rccl1) run bench_rccl1 300 env VBF_FORCE_PG=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 50 --no-cpu-baseline ;;
    residency) run pytest_residency 600 python -u -m pytest tests/test_gpu_residency.py -x -v -m gpu --timeout 120 --timeout-method thread ;;
    dist2)  run bench_dist2 300 env VBF_SHARE_DEVICE=1 VBF_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline ;;
    ubench) run ubench 300 ./tools/ubench ;;
    rdflat) run rdflat 300 ./tools/rdflat ;;
    pmcrdflat) (cd /tmp && run pmc_rdflat 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_rdflat" -o run -- "$ROOT/tools/rdflat") || exit $? ;;
    pmc2_5) (cd /tmp && run pmc2_5 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc2_5" -o run -- python3 "$ROOT/bench.py" --config 5 --steps 1 --warmup 1 --no-cpu-baseline --neg-keys 1000000) || exit $? ;;
    pmc3_5) (cd /tmp && run pmc3_5 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc3_5" -o run -- python3 "$ROOT/bench.py" --config 5 --steps 1 --warmup 1 --no-cpu-baseline --neg-keys 1000000) || exit $? ;;
    pmc2_3) (cd /tmp && run pmc2_3 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc2_3" -o run -- python3 "$ROOT/bench.py" --config 3 --steps 2 --warmup 1 --no-cpu-baseline --neg-keys 1000000) || exit $? ;;
    pmc3_3) (cd /tmp && run pmc3_3 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc3_3" -o run -- python3 "$ROOT/bench.py" --config 3 --steps 2 --warmup 1 --no-cpu-baseline --neg-keys 1000000) || exit $? ;;
    pmcsq3) (cd /tmp && run pmcsq3 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmcsq3" -o run -- python3 "$ROOT/bench.py" --config 3 --steps 2 --warmup 1 --no-cpu-baseline --neg-keys 1000000) || exit $? ;;
    abk1v2) run ab_k1v2_parity 900 env AB_PARITY=1 AB_ENVS="VBF_K1=2" bash tools/env_ab.sh
            run ab_k1v2_19 600 env AB_ENVS="VBF_K1=1 VBF_K1=2 VBF_K1=1 VBF_K1=2" AB_ARGS="--bits-per-key 19" bash tools/env_ab.sh
            run ab_k1v2_10 600 env AB_ENVS="VBF_K1=1 VBF_K1=2 VBF_K1=1 VBF_K1=2" bash tools/env_ab.sh ;;
    benchk) for b in 7 14 23; do run bench_k$b 300 python bench.py --no-cpu-baseline --bits-per-key $b --steps 20; done ;;
    benchkab) run ab_kclass 900 env AB_ENVS="VBF_KCLASS=0 VBF_KCLASS=1" AB_ARGS="--bits-per-key 7" bash tools/env_ab.sh
              run ab_kclass14 600 env AB_ENVS="VBF_KCLASS=0 VBF_KCLASS=1" AB_ARGS="--bits-per-key 14" bash tools/env_ab.sh
              run ab_kclass23 600 env AB_ENVS="VBF_KCLASS=0 VBF_KCLASS=1" AB_ARGS="--bits-per-key 23" bash tools/env_ab.sh
              run ab_kclass12 600 env AB_ENVS="VBF_KCLASS=0 VBF_KCLASS=1" AB_ARGS="--bits-per-key 12" bash tools/env_ab.sh ;;
    counters) (cd /tmp && run counters 120 rocprofv3 -L) || exit $? ;;
    pmc1) (cd /tmp && run pmc1 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc1" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline) || exit $? ;;
    pmc2) (cd /tmp && run pmc2 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc2" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline) || exit $? ;;
    pmc3) (cd /tmp && run pmc3 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc3" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline) || exit $? ;;
    pmcsq) (cd /tmp && run pmcsq 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmcsq" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline) || exit $? ;;
    pmc4) (cd /tmp && run pmc4 600 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY --output-format csv -d "$OUT/pmc4" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline) || exit $? ;;
    sstt)   run pytest_sst 300 python -u -m pytest tests/test_gpu_sst.py -x -v -m gpu --timeout 120 --timeout-method thread ;;
    k3sweep) run k3_sweep 900 bash tools/k3_sweep.sh ;;
    pmcsq19) (cd /tmp && run pmcsq19 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmcsq19" -o run -- python3 "$ROOT/bench.py" --bits-per-key 19 --steps 2 --warmup 1 --no-cpu-baseline) || exit $? ;;
    pmc2_19) (cd /tmp && run pmc2_19 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc2_19" -o run -- python3 "$ROOT/bench.py" --bits-per-key 19 --steps 2 --warmup 1 --no-cpu-baseline) || exit $? ;;
    pmc3_19) (cd /tmp && run pmc3_19 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc3_19" -o run -- python3 "$ROOT/bench.py" --bits-per-key 19 --steps 2 --warmup 1 --no-cpu-baseline) || exit $? ;;
    pmctcc) (cd /tmp && run pmctcc 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum --output-format csv -d "$OUT/pmctcc" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline) || exit $? ;;
    pmctcc19) (cd /tmp && run pmctcc19 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum --output-format csv -d "$OUT/pmctcc19" -o run -- python3 "$ROOT/bench.py" --bits-per-key 19 --steps 2 --warmup 1 --no-cpu-baseline) || exit $? ;;
    pmctcp) (cd /tmp && run pmctcp 600 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum --output-format csv -d "$OUT/pmctcp" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline) || exit $? ;;
    pmctcp19) (cd /tmp && run pmctcp19 600 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmctcp19" -o run -- python3 "$ROOT/bench.py" --bits-per-key 19 --steps 2 --warmup 1 --no-cpu-baseline) || exit $? ;;
    pmctcp10) (cd /tmp && run pmctcp10 600 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmctcp10" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline) || exit $? ;;
    abc16)  run ab_c16 900 env AB_PARITY=1 AB_ENVS="VBF_C16=1 VBF_C16=0" bash tools/env_ab.sh ;;
    abc16_19) run ab_c16_19 600 env AB_ENVS="VBF_C16=0 VBF_C16=1 VBF_C16=0 VBF_C16=1" AB_ARGS="--bits-per-key 19" bash tools/env_ab.sh ;;
    abc16_5) run ab_c16_5 600 bash -c 'for e in 0 1 0 1; do VBF_C16=$e python bench.py --config 5 --keys 250000000 --steps 5 --warmup 1 --no-cpu-baseline --neg-keys 1000000 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(\"C16=$e\", round(d[\"ms_per_step\"],3), \"ms\", round(d[\"build_kernel_ms\"],3))"; done' ;;
    prof19f) (cd /tmp && run prof19 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof19" -o run -- python3 "$ROOT/bench.py" --bits-per-key 19 --steps 40 --warmup 5 --no-cpu-baseline) || exit $? ;;
    prof)   (cd /tmp && run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 40 --warmup 5 --no-cpu-baseline) || exit $? ;;
  esac
done
echo "ALL DONE"
