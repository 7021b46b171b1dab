# variant: no L2 warm-up in the attention launch (att_prefetch never called)
p = "lm_kernels.hip"
s = open(p).read()
a = "      if (bx < sy.pf_n || bx < sy.pf_wo_n) att_prefetch(a, sy, bx);"
assert s.count(a) == 1
s = s.replace(a, "")
open(p, "w").write(s)
