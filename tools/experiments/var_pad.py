# variant: the round-4 device allocation sequence (the removed one-launch step / layer counter
# blocks allocated between the FFN and attention counter blocks again)
s = open("engine.hip").read()
a = "  RT_OK(alloc(&att_sync_, (size_t)Lc * kAttSyncInts));"
assert a in s
s = s.replace(a, "  { int* pad; RT_OK(alloc(&pad, (size_t)Lc * 88 * 64)); RT_OK(alloc(&pad, (size_t)Lc * 80 * 64)); }\n" + a)
open("engine.hip", "w").write(s)
