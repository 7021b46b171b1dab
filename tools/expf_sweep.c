#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <stdlib.h>
static uint64_t T[32];
static double asd(uint64_t u){double d;memcpy(&d,&u,8);return d;}
static uint64_t asu(double d){uint64_t u;memcpy(&u,&d,8);return u;}
static uint32_t asuf(float f){uint32_t u;memcpy(&u,&f,4);return u;}
static float asf(uint32_t u){float f;memcpy(&f,&u,4);return f;}
static float my_expf(float x, int variant){
  if (x == -INFINITY) return 0.0f;
  if (x != x) return x + x;
  if (x < -0x1.9fe368p6f) return 0.0f;
  double xd = x;
  const double InvLn2N = 0x1.71547652b82fep+0 * 32;
  const double SHIFT = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5/32/32/32, C1 = 0x1.ebfce50fac4f3p-3/32/32, C2=0x1.62e42ff0c52d6p-1/32;
  double z = InvLn2N * xd;
  double kd = z + SHIFT;
  uint64_t ki = asu(kd);
  kd -= SHIFT;
  double r = z - kd;
  if (variant==2) { r = fma(InvLn2N, xd, -kd); }
  uint64_t t = T[ki % 32];
  t += ki << (52 - 5);
  double s = asd(t);
  double zz, y, r2 = r*r;
  if (variant>=1) { zz = fma(C0, r, C1); y = fma(C2, r, 1.0); y = fma(zz, r2, y); }
  else { zz = C0*r + C1; y = C2*r + 1.0; y = zz*r2 + y; }
  y = y * s;
  return (float)y;
}
int main(){
  for (int i=0;i<32;i++){ long double v = powl(2.0L, i/32.0L); double d=(double)v; T[i]=asu(d)-((uint64_t)i<<47);}
  long mism[3]={0,0,0}; long n=0;
  /* all floats from -0 down to -104 */
  for (uint32_t u=0x80000000u; ; u++){
    float x=asf(u); if (x < -104.0f) break;
    float ref = expf(x);
    for (int v=0; v<3; v++){ float m=my_expf(x,v); if (asuf(m)!=asuf(ref)) { if (mism[v]<3) printf("v%d x=%a ref=%a mine=%a\n",v,x,ref,m); mism[v]++; } }
    n++;
  }
  printf("n=%ld mism v0=%ld v1=%ld v2=%ld\n", n, mism[0], mism[1], mism[2]);
  return 0;
}
