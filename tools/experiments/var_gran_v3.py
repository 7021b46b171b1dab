# debug: granule values used, but the value workgroup also waits for the K-slice counter (the key
# workgroup drains and arrives as in the slab form)
s = open("lm_kernels.hip").read()
a = """    if (!sy.gran) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && !sy.gran)"""
assert a in s
s = s.replace(a, """    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)""")
a = """                             __builtin_bit_cast(float, q[p][1][0]), __builtin_bit_cast(float, q[p][1][2])};
    }
    __syncthreads();"""
assert a in s
s = s.replace(a, """                             __builtin_bit_cast(float, q[p][1][0]), __builtin_bit_cast(float, q[p][1][2])};
    }
    sync_wait(sy.cnt + kSyncStride * (kLnReplicas + split), sy.key_per_slice, sy.err, 2, sy.opts);""")
open("lm_kernels.hip", "w").write(s)
