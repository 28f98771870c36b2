set -e
mkdir -p gpurun_out
for r in 1 2; do
  (cd .ab_old && timeout -k 10 200 python bench.py --steps 30 --warmup 3 --remote-steps 0 2>/dev/null) > gpurun_out/ab_old_$r.json
  timeout -k 10 200 python bench.py --steps 30 --warmup 3 --remote-steps 0 2>/dev/null > gpurun_out/ab_new_$r.json
done
