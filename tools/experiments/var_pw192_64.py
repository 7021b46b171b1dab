# variant: the 192-channel pointwise convs (stage 3 residual units' conv1) in 64-wide column tiles
# (80 VGPRs, 40 KB of LDS: three per CU leave room for a persistent decode workgroup), every other
# conv unchanged
s = open('codec.hip').read()
old = '''    if (K == 1 && Co % 96 == 0) TN = 96;'''
new = '''    if (K == 1 && Co % 96 == 0) TN = 96;
    if (K == 1 && Co == 192 && mode == 0) TN = 64;'''
assert old in s
s = s.replace(old, new)
open('codec.hip', 'w').write(s)
