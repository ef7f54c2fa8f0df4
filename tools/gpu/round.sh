#!/usr/bin/env bash
# One parameterised GPU-box script for the round's measurements (replaces the one-off rN*.sh scripts of rounds 1-5,
# in the git history). Usage on the box (via gpurun):  tools/gpu/round.sh TAG STEP [STEP ...]
# Each step runs under its own time limit and writes into gpurun_out/TAG/; the script stops at the first failure.
#   tests            GPU parity suite (pytest -m gpu)
#   tests:EXPR       GPU tests selected by pytest -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench            python bench.py (default shape) -> bench.json
#   bench_driver     python bench.py --steps 20 --warmup 5 -> bench_driver.json
#   slots1 / slots16 tools/processor_bench.py --only-slots at 1 / 16 threads (SRSGPU_BATCH_TIMING=1)
#   slots16ul        the same, UL only
#   slotslat         UL slot processors at 16 threads, free-running and paced at real time (500 us per slot and
#                    sector): throughput, PUSCH result latency, service plan / graph counters
#   dulowul          tools/du_low_bench.py, UL only, sector group with 13 symbols in flight, 4/6/8 sectors (latency)
#   slots_trace16    the same at 16 threads
#   slots_trace      rocprofv3 kernel + memory-copy trace of the slot processors at one thread (UL)
#   kstats           rocprofv3 --kernel-trace --stats of the default bench
#   lower            tools/lower_phy_bench.py with the multi-sector sweep
#   lower_trace      rocprofv3 kernel trace of the sector group at 8 sectors
#   dulow            tools/du_low_bench.py: lower PHY + PUSCH service per sector, paced, 1..8 sectors
#   lds              PMC pass of the bench: LDS issue stalls, bank conflicts, LDS-array cycles per kernel
#   traffic          FETCH_SIZE / WRITE_SIZE / SQ passes of the bench -> per-kernel HBM traffic vs algorithmic bytes
#                    (tools/chain_traffic.py), isolated kernel times, VALU issue and waits (tools/sq_summary.py)
#   ofdmab:DIR[:N]   tools/ofdm_bench.py (isolated OFDM launches, bench shape): in-tree library against DIR's, N rounds
#   hbm              tools/probes/hbm_rw.py: torch's fill / sum / copy rates (HBM write, read, copy ceilings)
#   ab:DIR[:N]       A/B of the default bench: the in-tree library against srsran-5g_amd/DIR's, N rounds
#   slotsab:V=X[:N]  A/B of the UL slot processors (16 threads): default environment against V=X, N rounds
#   benchab:V=X[:N]  A/B of the default bench: default environment against V=X, N rounds
set -o pipefail
TAG=${1:?tag}
shift
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  echo "== $step $(date +%T)"
  case "$step" in
    tests)
      timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
      tail -3 "$OUT/gpu_tests.log" ;;
    tests:*)
      timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        -k "${step#tests:}" > "$OUT/gpu_tests_k.log" 2>&1 || { tail -40 "$OUT/gpu_tests_k.log"; exit 1; }
      tail -3 "$OUT/gpu_tests_k.log" ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { cat "$OUT/smoke.log"; exit 1; }
      cat "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
      tail -c 600 "$OUT/bench.json" ;;
    bench_driver)
      timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" \
        || { tail -20 "$OUT/bench_driver.err"; exit 1; }
      tail -c 400 "$OUT/bench_driver.json" ;;
    slots1|slots16|slots16ul)
      T=${step#slots}; T=${T%ul}; DIRS=ul,dl; [[ "$step" == *ul ]] && DIRS=ul
      SRSGPU_BATCH_TIMING=1 timeout -k 10 400 python -u tools/processor_bench.py --only-slots --threads "$T" \
        --slots 100 --repetitions 3 --directions "$DIRS" > "$OUT/$step.json" 2> "$OUT/$step.log" \
        || { tail -20 "$OUT/$step.log"; exit 1; }
      grep -v '^pusch_slot_batch' "$OUT/$step.log" | tail -4; grep '^pusch_slot_batch' "$OUT/$step.log" | tail -2 ;;
    slotslat)
      SRSGPU_BATCH_TIMING=1 timeout -k 10 500 python -u tools/processor_bench.py --only-slots --threads 16 \
        --slots 100 --repetitions 3 --directions ul --pace-us 500 > "$OUT/slotslat.json" 2> "$OUT/slotslat.log" \
        || { tail -20 "$OUT/slotslat.log"; exit 1; }
      grep -v '^pusch_slot_batch' "$OUT/slotslat.log" | cut -c1-600 | tail -12 ;;
    dulowul)
      timeout -k 10 500 python -u tools/du_low_bench.py --direction ul --sectors 4,6,8 --variants group \
        --in-flight 13 > "$OUT/du_low_ul.json" 2> "$OUT/du_low_ul.log" || { tail -20 "$OUT/du_low_ul.log"; exit 1; }
      tail -c 1500 "$OUT/du_low_ul.json" ;;
    dulowdl)
      timeout -k 10 500 python -u tools/du_low_bench.py --direction dl --sectors 4,6,8 --variants alone,group \
        > "$OUT/du_low_dl.json" 2> "$OUT/du_low_dl.log" || { tail -20 "$OUT/du_low_dl.log"; exit 1; }
      tail -c 1500 "$OUT/du_low_dl.json" ;;
    slots_trace16)
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/trace16" -o slots -- python3 -u \
        tools/processor_bench.py --only-slots --threads 16 --repetitions 1 --slots 30 --directions ul \
        > "$OUT/slots_trace16.log" 2>&1 || { tail -20 "$OUT/slots_trace16.log"; exit 1; } ;;
    slots_trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/trace" -o slots -- python3 -u \
        tools/processor_bench.py --only-slots --threads 1 --repetitions 1 --slots 30 --directions ul \
        > "$OUT/slots_trace.log" 2>&1 || { tail -20 "$OUT/slots_trace.log"; exit 1; } ;;
    kstats)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kstats" -o k -- python3 -u bench.py \
        > "$OUT/kstats_bench.json" 2> "$OUT/kstats.log" || { tail -20 "$OUT/kstats.log"; exit 1; } ;;
    lower)
      echo "cgroup cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo n/a), nproc $(nproc)"
      timeout -k 10 400 python -u tools/lower_phy_bench.py --sectors 1,2,4,6,8,12 \
        --sweep-only cpu,gpu0,gpu4,gpu13,group0,group4,group13 > "$OUT/lower.json" 2> "$OUT/lower.log" \
        || { tail -20 "$OUT/lower.log"; exit 1; }
      tail -c 800 "$OUT/lower.json" ;;
    lower_trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/lower_trace" -o lower -- python3 -u \
        tools/lower_phy_bench.py --slots 100 --sectors 8 --sweep-only group4 > "$OUT/lower_trace.json" \
        2> "$OUT/lower_trace.log" || { tail -20 "$OUT/lower_trace.log"; exit 1; } ;;
    dulow)
      timeout -k 10 500 python -u tools/du_low_bench.py > "$OUT/du_low.json" 2> "$OUT/du_low.log" \
        || { tail -20 "$OUT/du_low.log"; exit 1; }
      tail -c 600 "$OUT/du_low.json" ;;
    lds)
      # LDS counters of the bench's kernels (one PMC pass): issue stalls on LDS, bank-conflict cycles, LDS-array cycles
      timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS \
        SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES -d "$OUT/pmc_lds" -o run --output-format csv -- python3 -u \
        bench.py --no-cpu-baseline --no-extra-points --no-extra-workloads --steps 40 --warmup 4 --min-time 0 \
        > "$OUT/pmc_lds.json" 2> "$OUT/pmc_lds.err" || { tail -20 "$OUT/pmc_lds.err"; exit 1; }
      CSV=$(find "$OUT/pmc_lds" -name "*counter_collection.csv" | head -1)
      python3 tools/pmc_summary.py "$CSV" > "$OUT/pmc_lds.txt"
      rm -rf "$OUT/pmc_lds"
      cat "$OUT/pmc_lds.txt" | cut -c1-400 ;;
    traffic)
      PB="--no-cpu-baseline --no-extra-points --no-extra-workloads --steps 40 --warmup 4 --min-time 0"
      timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv \
        -- python3 -u bench.py $PB > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err" || { tail -20 "$OUT/pmc_fetch.err"; exit 1; }
      timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv \
        -- python3 -u bench.py $PB > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err" || { tail -20 "$OUT/pmc_write.err"; exit 1; }
      timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY \
        SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS -d "$OUT/pmc_sq" -o run --output-format csv \
        -- python3 -u bench.py $PB > "$OUT/pmc_sq.json" 2> "$OUT/pmc_sq.err" || { tail -20 "$OUT/pmc_sq.err"; exit 1; }
      python3 tools/chain_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_fetch.json" > "$OUT/chain_traffic.json"
      SQ_CSV=$(find "$OUT/pmc_sq" -name "*counter_collection.csv" | head -1)
      python3 tools/sq_summary.py "$SQ_CSV" "$OUT/sq_valu.json" "$OUT/pmc_sq.json" > "$OUT/sq.log"
      find "$OUT" -name "*counter_collection.csv" -size +1M -delete
      find "$OUT" -name "*kernel_trace.csv" -delete
      cat "$OUT/sq.log" | head -14
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(k, round(v.get('traffic_ratio', 0), 3), round(v.get('isolated_us', 0), 1), round(v.get('hbm_fraction_of_8tbs_isolated', 0), 3)) for k, v in d['stages'].items()]" "$OUT/chain_traffic.json" ;;
    slotsab:*)
      # slotsab:VAR=V[,VAR2=V2][:N] — the UL slot processors at 16 threads (processor_bench.py --only-slots), N rounds
      # (default 2) alternating the default environment and the given variables
      SPEC=${step#slotsab:}; KV=${SPEC%%:*}; N=2; [[ "$SPEC" == *:* ]] && N=${SPEC##*:}
      IFS=, read -r -a VARS <<< "$KV"
      for i in $(seq 1 "$N"); do
        for v in default alt; do
          if [ "$v" = default ]; then E=(); else E=("${VARS[@]}"); fi
          env "${E[@]}" timeout -k 10 300 python -u tools/processor_bench.py --only-slots --threads 16 --slots 100 \
            --repetitions 3 --directions ul > "$OUT/slotsab_${v}_$i.json" 2> "$OUT/slotsab_${v}_$i.log" \
            || { tail -20 "$OUT/slotsab_${v}_$i.log"; exit 1; }
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], [(p['profile'][:12], [round(r['slots_per_s']) for r in p['runs']]) for p in d['slot_processors']['ul']])" \
            "$OUT/slotsab_${v}_$i.json" "$v ${E[*]}"
        done
      done ;;
    benchab:*)
      # benchab:VAR=V[,VAR2=V2][:N] — the default bench N rounds (default 2), alternating the default environment and
      # the given variables
      SPEC=${step#benchab:}; KV=${SPEC%%:*}; N=2; [[ "$SPEC" == *:* ]] && N=${SPEC##*:}
      IFS=, read -r -a VARS <<< "$KV"
      for i in $(seq 1 "$N"); do
        for v in default alt; do
          if [ "$v" = default ]; then E=(); else E=("${VARS[@]}"); fi
          env "${E[@]}" timeout -k 10 300 python -u bench.py > "$OUT/benchab_${v}_$i.json" 2> "$OUT/benchab_${v}_$i.err" \
            || { tail -20 "$OUT/benchab_${v}_$i.err"; exit 1; }
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), [round(p['value']) for p in d['operating_points']], round(d['stage_ms_per_step']['pusch_decode'], 4), {k: round(v['value']) for k, v in d.get('workloads', {}).items()})" \
            "$OUT/benchab_${v}_$i.json" "$v ${E[*]}"
        done
      done ;;
    hbm)
      timeout -k 10 120 python -u tools/probes/hbm_rw.py > "$OUT/hbm.json" 2>&1 || { tail -20 "$OUT/hbm.json"; exit 1; }
      tail -1 "$OUT/hbm.json" ;;
    ofdmab:*)
      SPEC=${step#ofdmab:}; DIR=${SPEC%%:*}; N=2; [[ "$SPEC" == *:* ]] && N=${SPEC##*:}
      for i in $(seq 1 "$N"); do
        for lib in lib "$DIR"; do
          echo "-- $lib"
          SRSGPU_LIB=srsran-5g_amd/$lib/libsrsgpu_phy.so timeout -k 10 120 python -u tools/ofdm_bench.py \
            > "$OUT/ofdmab_${lib}_$i.txt" 2>&1 || { tail -20 "$OUT/ofdmab_${lib}_$i.txt"; exit 1; }
          grep "ofdm_" "$OUT/ofdmab_${lib}_$i.txt" || true
        done
      done ;;
    setsweep)
      # the headline against the number of input sets in flight (bench.py --input-sets), two rounds
      for i in 1 2; do
        for n in 9 13 16 20 24; do
          timeout -k 10 200 python -u bench.py --input-sets "$n" --no-cpu-baseline --no-extra-points \
            --no-extra-workloads > "$OUT/setsweep_${n}_$i.json" 2> "$OUT/setsweep_${n}_$i.err" \
            || { tail -20 "$OUT/setsweep_${n}_$i.err"; exit 1; }
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('sets', sys.argv[2], round(d['value']))" \
            "$OUT/setsweep_${n}_$i.json" "$n"
        done
      done ;;
    ofdmsweep)
      # isolated OFDM launch time against the number of symbols per launch (slots x 4 ports x 14): the workgroup
      # rounds per CU show as steps in the time
      for s in 8 16 20 22 23 24 28 32 40 45 46 64; do
        timeout -k 10 120 python -u tools/ofdm_bench.py --slots "$s" --iters 100 > "$OUT/ofdmsweep_$s.txt" 2>&1 \
          || { tail -20 "$OUT/ofdmsweep_$s.txt"; exit 1; }
        echo "slots $s: $(head -2 "$OUT/ofdmsweep_$s.txt" | tr '\n' ' ')"
      done ;;
    ab:*)
      # ab:DIR[:N] — the default bench N times (default 2), alternating the in-tree library and srsran-5g_amd/DIR's
      SPEC=${step#ab:}; DIR=${SPEC%%:*}; N=2; [[ "$SPEC" == *:* ]] && N=${SPEC##*:}
      for i in $(seq 1 "$N"); do
        for lib in lib "$DIR"; do
          SRSGPU_LIB=srsran-5g_amd/$lib/libsrsgpu_phy.so timeout -k 10 300 python -u bench.py \
            > "$OUT/ab_${lib}_$i.json" 2> "$OUT/ab_${lib}_$i.err" || { tail -20 "$OUT/ab_${lib}_$i.err"; exit 1; }
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d.get('stage_ms_per_step', ''))" \
            "$OUT/ab_${lib}_$i.json" "$lib"
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
