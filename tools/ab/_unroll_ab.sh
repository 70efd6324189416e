set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/unr; mkdir -p $OUT
for v in base u16 u4 base u16; do
  if [ "$v" = base ]; then unset YSB_LIB_VARIANT; else export YSB_LIB_VARIANT=$v; fi
  rm -rf $OUT/$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- python3 $R/tools/bench_extra.py config3 --steps 10 --warmup 3 --segment 16666667 > $OUT/$v.json 2> $OUT/$v.err
  echo "$v $(grep -E 'rec_partition|rec_count' $OUT/$v/run_kernel_stats.csv | cut -d, -f1,4 | tr '\n' ' ') $(python3 -c "import json;d=json.load(open('$OUT/$v.json'));print(d['check']['truth_mismatched_cells'])")"
done
