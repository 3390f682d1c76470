// libm_f32_check.cpp — vloam-noted_amd/csrc/libm_f32.h (glibc's atanf / atan2f restated for
// the device) against the host's glibc on ~15M inputs: uniform lidar-range coordinates, random
// bit patterns (every exponent, NaN, inf, denormals), the special values, and ratios beyond
// 2^60.  Exit status 0 iff every result has glibc's bits.  Built with g++ (the __host__ /
// __device__ qualifiers defined away) and run by tests/test_host_models.py.
#include <cmath>
#include <cstdio>
#include <random>
#include <cstring>
#include "libm_f32.h"
using namespace loam;
static bool same(float a, float b){ int32_t x,y; memcpy(&x,&a,4); memcpy(&y,&b,4); return x==y || (a!=a && b!=b);}
int main(){
  std::mt19937_64 g(1); long bad=0, n=0;
  auto chk=[&](float y,float x){ n++; float a=glibc_atan2f(y,x), b=atan2f(y,x); if(!same(a,b)){ if(bad<10) printf("atan2 y=%a x=%a mine=%a glibc=%a\n",y,x,a,b); bad++;} };
  auto chk1=[&](float x){ n++; float a=glibc_atanf(x), b=atanf(x); if(!same(a,b)){ if(bad<10) printf("atan x=%a mine=%a glibc=%a\n",x,a,b); bad++;} };
  std::uniform_real_distribution<float> U(-120.f,120.f);
  for(int i=0;i<5000000;i++){ chk(U(g),U(g)); }
  for(int i=0;i<3000000;i++){ uint32_t w=(uint32_t)g(); float f; memcpy(&f,&w,4); chk1(f); uint32_t w2=(uint32_t)g(); float f2; memcpy(&f2,&w2,4); chk(f,f2);}
  float sp[]={0.f,-0.f,1.f,-1.f,INFINITY,-INFINITY,NAN,1e-30f,-1e-30f,1e30f,3.f,0.5f};
  for(float a:sp) for(float b:sp){ chk(a,b); chk1(a);}
  for(int i=0;i<2000000;i++){ float x=U(g); chk(x*1e-20f, U(g)); chk(U(g), x*1e-20f);}
  printf("checked %ld, mismatches %ld\n", n, bad); return bad!=0;
}
