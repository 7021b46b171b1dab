# debug: pure granule form + the key workgroup drains its stores before the key-done arrival
s = open("lm_kernels.hip").read()
a = """    if (!sy.gran) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");"""
assert a in s
s = s.replace(a, """    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");""")
open("lm_kernels.hip", "w").write(s)
