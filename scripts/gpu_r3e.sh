#!/bin/bash
# Fused write kernel (no SDMA copy on the write path) + durable-name A/B next to the sweep.
set -o pipefail
out=gpurun_out/r3e
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu \
  > $out/pytest_kernels.log 2>&1 || { tail -30 $out/pytest_kernels.log; exit 1; }
tail -2 $out/pytest_kernels.log
DFS_FUSED_WRITE=1 timeout -k 10 300 build/native/io_bench --no-fsync --iters 30 --dir /tmp/iobf1 > $out/io_fused1.json 2> $out/io_fused1.err && \
DFS_FUSED_WRITE=0 timeout -k 10 300 build/native/io_bench --no-fsync --iters 30 --dir /tmp/iobf0 > $out/io_fused0.json 2> $out/io_fused0.err || exit $?
rm -rf /tmp/iobf1 /tmp/iobf0
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$OLDPWD/$out/prof_io" -o io -- "$OLDPWD/build/native/io_bench" --no-fsync --iters 10 --dir /tmp/iobp) \
   > $out/io_prof.json 2> $out/io_prof.err || exit $?
sweep() { timeout -k 10 120 build/native/io_bench --disk-sweep --dir /tmp/iob --cases "10:0,10:0" > $out/sweep_$1.json 2>&1; }
one() { DFS_FINAL_NAMES=$1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --remote-steps 0 > $out/bench_fn$1_$2.json 2> $out/bench_fn$1_$2.err; }
sweep a && one 1 a && one 0 a && one 1 b && one 0 b && sweep b || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --remote-steps 3 --profile-dir $out/prof > $out/bench_prof.json 2> $out/bench_prof.err || exit $?
python scripts/marker_phases.py $out/prof > $out/marker_phases.txt; cat $out/marker_phases.txt
python -c "
import csv,glob
for f in glob.glob('$out/prof*/**/*kernel_stats.csv', recursive=True):
    print(f)
    for r in csv.DictReader(open(f)): print('  ', r['Name'][:70], r['Calls'], r['AverageNs'])
"
for f in $out/sweep_a.json $out/bench_fn1_a.json $out/bench_fn0_a.json $out/bench_fn1_b.json $out/bench_fn0_b.json $out/sweep_b.json $out/bench_prof.json; do
  echo "== $f"; python -c "import json,sys; d=json.load(open('$f')); print({k: d[k] for k in ('value','write_mb_per_s','read_mb_per_s','write_p50_ms','client_phase_p50_ms_rank0','host_cpu_util_rank0') if k in d} if 'value' in d else d)"
done
python -c "
import json
for m in (1, 0):
    d = json.load(open('$out/io_fused%d.json' % m))
    print('fused', m, {k: v for k, v in d.items() if 'write' in k})
"
