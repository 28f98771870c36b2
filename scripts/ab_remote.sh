# Same-box A/B of the remote-client phase (native gRPC client + servers): .ab_old (a built
# worktree of the baseline commit) vs this tree, alternating, two runs each.
set -e
mkdir -p gpurun_out
for r in 1 2; do
  (cd .ab_old && timeout -k 10 300 python bench.py --steps 2 --warmup 1 --remote-steps 6 2>/dev/null) > gpurun_out/abr_old_$r.json
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --remote-steps 6 2>/dev/null > gpurun_out/abr_new_$r.json
done
