"""Data-path compute ops: CRC-32 (K1/K2/K3) and Reed-Solomon (K4/K5), each with a CDNA4
HIP implementation (csrc/gpu_kernels.hip, driven through the HBM ChunkStore) and a native
CPU implementation (PCLMUL CRC, table GF(2^8)) used when no GPU is present."""
