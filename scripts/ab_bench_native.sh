#!/bin/bash
# Same-box A/B of this session's read/write-path changes, alternating to cancel the
# volume's drift:
#   base: Python thread-pool benchmark workers (DFS_BENCH_NATIVE=0), 8 MD5 workers, and
#         reads as verify kernel + SDMA copy (DFS_FUSED_READ=0) — the previous defaults
#   nat:  native benchmark worker threads, 16 MD5 workers
#   all:  nat + the fused K3 verify+copy read kernel (the new defaults)
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/ab_native
run() {  # tag native hash fused durability
  DFS_BENCH_NATIVE=$2 DFS_HASH_THREADS=$3 DFS_FUSED_READ=$4 timeout -k 10 300 python bench.py --steps 10 --warmup 2 \
    --remote-steps 2 --durability "$5" > "gpurun_out/ab_native/$1.json" 2> "gpurun_out/ab_native/$1.err"
}
for rep in 1 2; do
  run "base_nvme_$rep" 0 8 0 nvme-sync && run "nat_nvme_$rep" 1 16 0 nvme-sync && \
  run "all_nvme_$rep" 1 16 1 nvme-sync || exit $?
done
run base_hbm 0 8 0 hbm-ack && run all_hbm 1 16 1 hbm-ack || exit $?
echo ab_native done
