# The structural index's classification alone (YSB_DIAG_FLAT_IDX) against the flat tier's whole
# parse (no probe, no count) and Phase A alone, layout 2 forced, mixed and reordered producers.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-r6m}
mkdir -p $out
for leg in mixed_flat_fixed reorder_flat_fixed; do
  for v in none fidx flatnj diag; do
    vv=$v; [ $v = none ] && vv=""
    YSB_LIB_VARIANT=$vv timeout -k 10 200 python tools/extra_one.py $leg --extra-steps 10 --warmup 3 > $out/${leg}_$v.json 2> $out/${leg}_$v.err || { tail -3 $out/${leg}_$v.err; exit 2; }
    python -c "import json; r=json.loads(open('$out/${leg}_$v.json').read().strip().splitlines()[-1]); print('$leg', '$v', r['avg_launch_ms'], r['events_per_s']/1e9)"
  done
done
for v in none fidx; do
  vv=$v; [ $v = none ] && vv=""
  YSB_LIB_VARIANT=$vv timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH --output-format csv -d $out/pmc_$v -o run -- python3 tools/extra_one.py mixed_flat_fixed --extra-steps 2 --warmup 1 > $out/pmc_$v.json 2> $out/pmc_$v.err || exit 3
  find $out/pmc_$v -name "*counter_collection.csv" | head -1 | xargs -I{} cp {} $out/sq_$v.csv
  rm -rf $out/pmc_$v
done
