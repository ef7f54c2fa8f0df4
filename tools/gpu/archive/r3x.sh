# Round 3: PDSCH encoder TB CRC inline (carrier codeblock's workgroup) vs the separate tb_crc_kernel, headline bench A/B.
set -o pipefail
OUT=gpurun_out/r3x
mkdir -p $OUT
B="--no-extra-workloads --no-extra-points --no-cpu-baseline --warmup 20"
for i in 1 2; do
  for f in 1 0; do
    SRSGPU_ENCODER_TB_CRC_INLINE=$f timeout -k 10 200 python bench.py $B > $OUT/inline${f}_$i.json 2> $OUT/inline${f}_$i.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']), round(d['stage_ms_per_step']['pdsch_encode']*1e3,1))" $OUT/inline${f}_$i.json
  done
done
