# variant: the vocoder co-residency policy (kCodecResv) from the environment VAR_RESV
import os
p = "codec.hip"
s = open(p).read()
a = "constexpr int kCodecResv = 2;"
assert s.count(a) == 1
s = s.replace(a, "constexpr int kCodecResv = %d;" % int(os.environ["VAR_RESV"]))
open(p, "w").write(s)
