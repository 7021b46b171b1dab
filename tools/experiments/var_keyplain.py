# variant: the persistent FFN launch's key partial slabs stored with plain 16-byte stores (the line
# stays in the XCD's L2) instead of write-through sc1 stores (which drop it): the value workgroups that
# read them run on the same XCD (consumer-aligned grid), so their sc1 loads hit that L2
p = "lm_kernels.hip"
s = open(p).read()
def rep(a, b):
    global s
    assert s.count(a) == 1, a[:60]
    s = s.replace(a, b)
rep("        store_wt(rs, (int)(o * 4), v);", """        if (a.wt == 2) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_, v), rs, (int)(o * 4), 0, 0);
        else store_wt(rs, (int)(o * 4), v);""")
rep("ka.xmap = 2; ka.ntiles = kt; ka.wt = 1;", "ka.xmap = 2; ka.ntiles = kt; ka.wt = 2;")
open(p, "w").write(s)
