#!/bin/bash
# Copies a round's GPU evidence (tools/round_final.sh parts a and b) from gpurun_out/ into
# profiles/ under one prefix:   tools/collect_profiles.sh TAG_A TAG_B PREFIX   (e.g. r5a r5b r05)
set -euo pipefail
A=gpurun_out/$1; B=gpurun_out/$2; P=profiles/$3
tail -1 $A/bench.json > ${P}_bench.json
cp $A/trace/run_kernel_stats.csv ${P}_kernel_stats.csv
cp $A/scan_launches.txt ${P}_scan_launches.txt
{ echo "# headline scan_kernel<false, false, false, 0>: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ($A, tools/final_profile.sh)"
  python3 tools/pmc_summary.py $A "scan_kernel<false, false, false, 0>"; } > ${P}_pmc_summary.txt
cp $B/c3trace/run_kernel_stats.csv ${P}_config3_kernel_stats.csv
{ echo "# configs[2] (tools/extra_one.py config3): the record-mode scan, then the record kernels ($B/c3pmc)"
  python3 tools/pmc_summary.py $B/c3pmc "scan_kernel<true, false, true, 0>"
  echo "## record-mode kernels"; python3 tools/pmc_summary.py $B/c3pmc "rec_"; } > ${P}_config3_pmc.txt
cp $B/rawtrace/run_kernel_stats.csv ${P}_raw_kernel_stats.csv
tail -1 $B/rawtrace.json > ${P}_raw_dropin.json
cp $B/mixtrace/run_kernel_stats.csv ${P}_mixed_kernel_stats.csv
cp $B/streamtrace/run_kernel_stats.csv ${P}_stream_kernel_stats.csv
tail -1 $B/streamtrace.json > ${P}_stream_native_trace_run.json   # the runner itself under the tracer
cp $B/xtrace/run_kernel_stats.csv ${P}_exchange_kernel_stats.csv
tail -1 $B/xcost.json > ${P}_exchange_cost.json
{ echo "# SQ counters per flat-tier dispatch (tools/sq_passes.sh over tools/extra_one.py reorder_flat_fixed, $B/sq_flat)"
  python3 tools/pmc_summary.py $B/sq_flat "scan_kernel<false, false, false, 2>"
  echo; echo "## four producers interleaved line by line (mixed_flat_fixed, $B/sq_mix)"
  python3 tools/pmc_summary.py $B/sq_mix "scan_kernel<false, false, false, 2>"; } > ${P}_flat_sq.txt
echo "collected into ${P}_*"
