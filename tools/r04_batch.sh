#!/bin/bash
# Round-4 measurement batch: exchange serial vs overlapped, PMC traffic of the
# exchange-form kernel, workloads R (device episodes), F (full tree), D.
set -o pipefail
O=gpurun_out/${TAG:-r04c}; mkdir -p $O
export TMPDIR=/tmp
TAG=$TAG bash tools/xchg_ab.sh 2 || exit 1
for w in R F D; do
  echo "[batch] $w $(date +%T)" >&2
  timeout -k 10 300 python bench.py --cpu-seconds 0 --no-second-pass --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -5 $O/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/bench_$w.json') if l.startswith('{')][0]); print('$w', d['value'], d['unit'], 'ms/step', d['ms_per_step'], (d.get('roofline') or {}).get('frac'))"
done
echo "[batch] timelines $(date +%T)" >&2
timeout -k 10 150 python tools/chain_timeline.py run 100000 3 > $O/timeline_B.txt 2>&1 || { echo "timeline B failed"; tail -5 $O/timeline_B.txt; exit 1; }
grep -v '^JSON' $O/timeline_B.txt | tail -4
timeout -k 10 150 python tools/chain_timeline.py run 1000000 10 > $O/timeline_C.txt 2>&1 || { echo "timeline C failed"; tail -5 $O/timeline_C.txt; exit 1; }
grep -v '^JSON' $O/timeline_C.txt | tail -4
echo "[batch] pmc $(date +%T)" >&2
TAG=$TAG/pmc_xchg ARGS="1000000 10 xchg 20 4" bash tools/pmc.sh > $O/pmc.log 2>&1 &&
python tools/pmc_summary.py $O/pmc_xchg $O/traffic_chain_xchg.json 160e6 "k_episode_chain<1, 2, 3" "k_episode_chain[exchange]"
