# variant: k_gemm_wide with LDS-only barriers around the store staging and at the loop end
s = open('lm_kernels.hip').read()
a = s.index('void k_gemm_wide(GemmArgs a)'); b = s.index('tl_end(a.tl);', a)
seg = s[a:b]
seg = seg.replace('''    __syncthreads();  // every wave is done reading its X fragments''', '''    lds_barrier();  // every wave is done reading its X fragments''')
seg = seg.replace('''          st[(m * 16 + 4 * g + jj) * LDT + j * 64 + wave * 16 + li] = acc_h[j][m][jj] + acc_l[j][m][jj];
    __syncthreads();''', '''          st[(m * 16 + 4 * g + jj) * LDT + j * 64 + wave * 16 + li] = acc_h[j][m][jj] + acc_l[j][m][jj];
    lds_barrier();''')
seg = seg.replace('''    __syncthreads();  // every wave is done with the LDS X image / store staging''', '''    lds_barrier();  // every wave is done with the LDS X image / store staging''')
assert seg.count('lds_barrier') == 3
s = s[:a] + seg + s[b:]
helper = '__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_barrier" ::: "memory"); }\n'
anchor = '// Prefill (multi-row) planes GEMMs of one segment'
s = s.replace(anchor, helper + anchor)
open('lm_kernels.hip', 'w').write(s)
