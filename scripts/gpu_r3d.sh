#!/bin/bash
# Durable writes to final names (fresh ids) next to the volume's sweep, A/B/A; remote tail
# after the reply-pool prewarm (bench remote phase + roctx phases of the chunkserver).
set -o pipefail
out=gpurun_out/r3d
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -m gpu \
  > $out/pytest_kernels.log 2>&1 || { tail -30 $out/pytest_kernels.log; exit 1; }
tail -2 $out/pytest_kernels.log
sweep() { timeout -k 10 120 build/native/io_bench --disk-sweep --dir /tmp/iob --cases "10:0,10:0" > $out/sweep_$1.json 2>&1; }
one() { timeout -k 10 300 python bench.py --steps 20 --warmup 5 --remote-steps 5 > $out/bench_$1.json 2> $out/bench_$1.err; }
sweep a && one a && sweep b && one b && sweep c || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --remote-steps 5 --profile-dir $out/prof > $out/bench_prof.json 2> $out/bench_prof.err || exit $?
python scripts/marker_phases.py $out/prof > $out/marker_phases.txt; cat $out/marker_phases.txt
for f in $out/sweep_a.json $out/bench_a.json $out/sweep_b.json $out/bench_b.json $out/sweep_c.json $out/bench_prof.json; do
  echo "== $f"; python -c "import json,sys; d=json.load(open('$f')); print({k: d[k] for k in ('value','write_mb_per_s','read_mb_per_s','write_p50_ms','client_phase_p50_ms_rank0','remote_client') if k in d} if 'value' in d else d)"
done
