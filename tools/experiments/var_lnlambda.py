# variant: ln1024_body's LayerNorm as its own lambda again (round-4 code) instead of ln1024_apply
s = open("lm_kernels.hip").read()
a = "  auto ln = [&](float4_& x, int slot_base) { ln1024_apply(x, w, b, red, slot_base); };"
b = """  auto ln = [&](float4_& x, int slot_base) {
    const float mean = block_sum_1b((x[0] + x[1]) + (x[2] + x[3]), red, slot_base) * (1.0f / C);
    const float4_ d = x - mean;
    const float var = block_sum_1b((d[0] * d[0] + d[1] * d[1]) + (d[2] * d[2] + d[3] * d[3]), red, slot_base + 1) * (1.0f / C);
    const float rstd = 1.0f / sqrtf(var + 1e-5f);
    x = d * rstd * w + b;
  };"""
assert a in s
s = s.replace(a, b)
open("lm_kernels.hip", "w").write(s)
