#!/bin/bash
# Copy one gpu_profile.sh session's results into profiles/ (tracked): bench lines, rocprofv3
# kernel-stats CSVs and the timed-region summaries. Usage: bash tools/sessions/collect_profiles.sh <tag> <round-prefix>
set -eu
cd "$(dirname "$0")/../.."
TAG=$1; PFX=$2
SRC=gpurun_out/$TAG
for f in "$SRC"/bench_*.json; do
  c=$(basename "$f" .json | sed 's/^bench_//')
  cp "$f" "profiles/${PFX}_bench_${c}.json"
  case $c in C5) w=3; s=20;; C4) w=3; s=30;; C3) w=10; s=100;; *) w=20; s=200;; esac
  if [ -d "$SRC/prof_$c" ]; then
    cp "$SRC/prof_$c/run_kernel_stats.csv" "profiles/${PFX}_${c}_rocprof_kernel_stats.csv"
    python tools/rocprof_summary.py "$SRC/prof_$c" --log "$SRC/rocprof_$c.log" > "profiles/${PFX}_${c}_rocprof_timed_region.txt"
  fi
done
ls profiles | grep "^${PFX}_"
