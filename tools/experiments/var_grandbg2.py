# debug variant: the pure granule form, the first value workgroup of layers 0 and 1 printing the
# tag it waits for and what its lane 0 found
s = open("lm_kernels.hip").read()
a = """        if (__all(ok)) break;
        __builtin_amdgcn_s_sleep(1);"""
b = """        if (__all(ok)) break;
        if (bx == 0 && sy.layer < 2 && lane == 0 && (__builtin_amdgcn_s_memrealtime() - t0) < 3)
          printf("GRANDBG2 layer %d tag %u found %u data %08x (polling)\\n", sy.layer, tag, q[0][0][1], q[0][0][0]);
        __builtin_amdgcn_s_sleep(1);"""
assert a in s; s = s.replace(a, b)
a = """#pragma unroll
      for (int p = 0; p < NX; ++p)
        xr[p][0] = (float4_){__builtin_bit_cast(float, q[p][0][0]), __builtin_bit_cast(float, q[p][0][2]),"""
b = """      if (bx == 0 && sy.layer < 2 && lane == 0)
        printf("GRANDBG2 layer %d split %d kbeg %d tag %u found %u data %08x\\n", sy.layer, split, kbeg, tag, q[0][0][1], q[0][0][0]);
#pragma unroll
      for (int p = 0; p < NX; ++p)
        xr[p][0] = (float4_){__builtin_bit_cast(float, q[p][0][0]), __builtin_bit_cast(float, q[p][0][2]),"""
assert a in s; s = s.replace(a, b)
open("lm_kernels.hip", "w").write(s)
