# debug: pure granule form + the key workgroup also stores its partial slab
s = open("lm_kernels.hip").read()
a = """    if (g == 0 && col < Nn) gran_store(sy.gran + (int64_t)split * sy.gran_ld + col_off + col, result(0, 0), gran_tag(sy));
  } else if (a.wt) {"""
assert a in s
s = s.replace(a, """    if (g == 0 && col < Nn) gran_store(sy.gran + (int64_t)split * sy.gran_ld + col_off + col, result(0, 0), gran_tag(sy));
  }
  if (a.wt) {""")
open("lm_kernels.hip", "w").write(s)
