# variant: the attention launch's L2 warm-up hold (kHoldPf) from the environment VAR_PF (10 ns ticks)
import os
p = "lm_kernels.hip"
s = open(p).read()
a = "constexpr int kHoldPf = 300;"
assert s.count(a) == 1
s = s.replace(a, "constexpr int kHoldPf = %d;" % int(os.environ["VAR_PF"]))
open(p, "w").write(s)
