# variant (timing only): value / Wo workgroups take their work_done stamp once X is staged in LDS
# (before the MFMAs and the epilogue) -- splits the X hand-off latency from the compute
s = open("lm_kernels.hip").read()
a = "  __syncthreads();\n  const int rg_next = rg + (int)gridDim.z;"
assert a in s
s = s.replace(a, "  __syncthreads();\n  if constexpr (ROLE == 2 || ROLE == 4) sync_stamp(sy, 2);\n  const int rg_next = rg + (int)gridDim.z;")
b = "  if constexpr (ROLE != 0) sync_stamp(sy, 2);"
assert b in s
s = s.replace(b, "  if constexpr (ROLE != 0 && ROLE != 2 && ROLE != 4) sync_stamp(sy, 2);")
open("lm_kernels.hip", "w").write(s)
