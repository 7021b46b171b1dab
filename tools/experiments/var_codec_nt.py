# variant: the vocoder's activation streams marked non-temporal (window loads into LDS with the nt
# cache-policy bit, residual loads and every epilogue store nontemporal): planes of up to 2 GB never
# hit in the Infinity Cache, and may then leave the decode's hand-off lines there
s = open('codec.hip').read()
old1 = '''        if (b >= WRp / 16) __builtin_amdgcn_raw_ptr_buffer_load_lds(rxl, dst, 16, voff[u], aso, 0, 0);
        else __builtin_amdgcn_raw_ptr_buffer_load_lds(rxh, dst, 16, voff[u], aso, 0, 0);'''
new1 = '''        if (b >= WRp / 16) __builtin_amdgcn_raw_ptr_buffer_load_lds(rxl, dst, 16, voff[u], aso, 0, 2);
        else __builtin_amdgcn_raw_ptr_buffer_load_lds(rxh, dst, 16, voff[u], aso, 0, 2);'''
assert old1 in s; s = s.replace(old1, new1)
old2 = '''    if (a.res && q < Tin) rv[it] = *(const float4_*)(a.res + yoff + (int64_t)(q * ostr + phase) * a.Co + co0 + c4);'''
new2 = '''    if (a.res && q < Tin) rv[it] = __builtin_nontemporal_load((const float4_*)(a.res + yoff + (int64_t)(q * ostr + phase) * a.Co + co0 + c4));'''
assert old2 in s; s = s.replace(old2, new2)
old3 = '''      else v += *(const float4_*)(a.res + o);
    }
    if (a.y) *(float4_*)(a.y + o) = v;'''
new3 = '''      else v += __builtin_nontemporal_load((const float4_*)(a.res + o));
    }
    if (a.y) __builtin_nontemporal_store(v, (float4_*)(a.y + o));'''
assert old3 in s; s = s.replace(old3, new3)
old4 = '''      *(uint2*)(a.yh + op) = make_uint2(h01, h23);
      *(uint2*)(a.yl + op) = make_uint2(l01, l23);
    }
  }
  }
}'''
new4 = '''      typedef uint32_t u32v2 __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store((u32v2){h01, h23}, (u32v2*)(a.yh + op));
      __builtin_nontemporal_store((u32v2){l01, l23}, (u32v2*)(a.yl + op));
    }
  }
  }
}'''
assert old4 in s; s = s.replace(old4, new4)
open('codec.hip', 'w').write(s)
