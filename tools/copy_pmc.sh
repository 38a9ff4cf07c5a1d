#!/bin/bash
# copy a tools/pmc_general.sh / pmc_variants.sh output directory's counter CSVs, kernel stats and summary into profiles/
#   tools/copy_pmc.sh gpurun_out/pmc_gen profiles/r06_pmc_gen
set -e
src=$1; dst=$2
mkdir -p "$dst"
for d in "$src"/*/; do
  n=$(basename "$d")
  [ -f "$d/run_counter_collection.csv" ] && cp "$d/run_counter_collection.csv" "$dst/$n.csv"
  [ -f "$d/run_kernel_stats.csv" ] && cp "$d/run_kernel_stats.csv" "$dst/${n}_kernel_stats.csv"
done
[ -f "$src/summary.txt" ] && cp "$src/summary.txt" "$dst/summary.txt"
ls "$dst" | wc -l
