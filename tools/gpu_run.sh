#!/bin/bash
# One launcher for GPU-box work (replaces the per-round gpu_r0N*.sh one-offs). Run it through gpurun:
#
#   gpurun -- 'bash tools/gpu_run.sh OUT STEP [STEP ...]'
#
# OUT is a directory under gpurun_out/; each STEP runs under its own time limit, writes its output
# under OUT, and the script stops at the first step that fails (no GPU work after a failed, killed
# or timed-out step). Steps:
#   tests[:-k expr]    GPU test suite (pytest -m gpu), optionally a -k subset
#   smoke              __graft_entry__.smoke()
#   bench              bench.py default line (N=1)
#   configs            tools/bench_configs.py C2 C2L C2LN C3 C4 C5
#   groups             tools/bench_groups.py GROUP BY cardinality sweep at 1B rows
#   tripdata           tools/bench_tripdata.py (the reference's own query, K:1336)
#   fp64               tools/exp_fp64_sum.py C5 C4 (exact vs opt-in fast fp64 sums)
#   profile            profiles/run_profile.sh (bench kernel trace + PMC traffic)
#   c3pmc              tools/prof_c3_pmc.sh (C3 kernel trace, FETCH/WRITE, SQ and TA counters)
#   c2prof             tools/prof_c2.sh with CFG=C2 (C2 kernel trace + counters)
#   prof_trip          tools/prof_tripdata.sh (tripdata kernel trace)
#   prof_fp64          tools/prof_fp64_sum.sh (C5 trace + SQ / LDS counters per mode)
#   fxq                tools/exp_fxq.sh (exact-sum kernel code-shape A/B on C5)
#   spill              tools/exp_spill.sh (spilling pass reach past the compact table, QE_SPILL_MAXPCT)
#   csvpmc             tools/prof_csv_pmc.sh (SQ / LDS counters of the tripdata kernels, 4M rows)
#   triptraffic        tools/prof_trip_traffic.sh (FETCH_SIZE / WRITE_SIZE of the tripdata kernels)
#   env:NAME=VALUE     set an environment variable for the following steps (env:TAG=x suffixes the
#                      output files of tripdata / configs / fp64 with _x)
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/${1:?usage: gpu_run.sh OUT STEP...}
shift
mkdir -p "$OUT"
T="timeout -k 10"
step() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  echo "== $name $(date +%T)" >> "$OUT/steps.log"
  if ! $T "$lim" "$@"; then
    echo "   FAILED (rc=$?)" >> "$OUT/steps.log"
    exit 1
  fi
}
for s in "$@"; do
  case "$s" in
    env:*) export "${s#env:}" ;;
    tests) step tests 1000 bash -c "python3 -u -m pytest tests -q -m gpu --timeout 280 --timeout-method thread > '$OUT/tests.txt' 2>&1" ;;
    tests:*) step tests 1000 bash -c "python3 -u -m pytest tests -q -m gpu --timeout 280 --timeout-method thread -k '${s#tests:}' > '$OUT/tests.txt' 2>&1" ;;
    smoke) step smoke 180 bash -c "python3 -c 'import __graft_entry__ as g; g.smoke()' > '$OUT/smoke.txt' 2>&1" ;;
    bench) step bench 300 bash -c "python3 bench.py > '$OUT/bench.json' 2> '$OUT/bench.err'" ;;
    configs) step configs 600 bash -c "python3 tools/bench_configs.py C2 C2L C2LN C3 C4 C5 > '$OUT/configs${TAG:+_$TAG}.jsonl' 2> '$OUT/configs${TAG:+_$TAG}.err'" ;;
    groups) step groups 600 bash -c "python3 tools/bench_groups.py 1000000000 1024 4096 5800 8192 65536 1048576 > '$OUT/groups.jsonl' 2> '$OUT/groups.err'" ;;
    tripdata) step tripdata 300 bash -c "python3 tools/bench_tripdata.py > '$OUT/tripdata${TAG:+_$TAG}.json' 2> '$OUT/tripdata${TAG:+_$TAG}.err'" ;;
    fp64) step fp64 300 bash -c "python3 tools/exp_fp64_sum.py C5 C4 --rounds 3 > '$OUT/fp64${TAG:+_$TAG}.jsonl' 2>&1" ;;
    csvpmc) step csvpmc 700 env ROWS=4000000 bash tools/prof_csv_pmc.sh ;;
    triptraffic) step triptraffic 700 env ROWS=4000000 bash tools/prof_trip_traffic.sh ;;
    profile) step profile 600 bash profiles/run_profile.sh ;;
    prof_trip) step prof_trip 500 env ROWS=4000000 bash tools/prof_tripdata.sh ;;
    prof_fp64) step prof_fp64 600 bash tools/prof_fp64_sum.sh ;;
    fxq) step fxq 900 bash tools/exp_fxq.sh ;;
    c3pmc) step c3pmc 900 bash tools/prof_c3_pmc.sh ;;
    c2prof) step c2prof 600 env CFG=C2 bash tools/prof_c2.sh ;;
    spill) step spill 1100 bash tools/exp_spill.sh ;;
    *) echo "unknown step $s" >> "$OUT/steps.log"; exit 2 ;;
  esac
done
echo "== done $(date +%T)" >> "$OUT/steps.log"
