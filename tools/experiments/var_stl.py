# variant (timing only): value workgroups stamp work_done once their X loads have landed (thread 0's
# wave, s_waitcnt vmcnt(0) right after the loads), Wo likewise
s = open("lm_kernels.hip").read()
a = """    sync_wait(sy.cnt + kSyncStride * (kLnReplicas + split), sy.key_per_slice, sy.err, 2, sy.opts);
    sync_stamp(sy, 1);
    load_x();"""
assert a in s
s = s.replace(a, a + """
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sync_stamp(sy, 2);""")
b = "  if constexpr (ROLE != 0) sync_stamp(sy, 2);"
assert b in s
s = s.replace(b, "  if constexpr (ROLE != 0 && ROLE != 2) sync_stamp(sy, 2);")
open("lm_kernels.hip", "w").write(s)
