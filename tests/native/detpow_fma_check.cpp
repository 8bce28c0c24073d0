// det_pow<true> (FMA exact products, the device's variation operators) against det_pow<>
// (Dekker's split, restated by oracle/device_order.py det_pow): bit-identical on the SBX and
// polynomial-mutation argument domains.  Built and run by tests/test_detpow_cpu.py.
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <cmath>
#include "detmath.h"
using namespace mv;
static uint64_t bits(double d){uint64_t u; std::memcpy(&u,&d,8); return u;}
int main(){
  std::mt19937_64 g(7); std::uniform_real_distribution<double> U(0.0,1.0);
  long bad=0, n=0;
  auto chk=[&](double x,double y){ double a=det_pow<false>(x,y), b=det_pow<true>(x,y); ++n; if(bits(a)!=bits(b)){ if(bad<10) printf("x=%.17g y=%.17g %.17g %.17g\n",x,y,a,b); ++bad;} };
  for(long i=0;i<500000;++i){
    double r=U(g);
    // SBX alpha: beta >= 1 (up to 1e9), y = -31
    double beta = 1.0 + std::pow(10.0, 9.0*U(g)) * (U(g)<0.3 ? 1e-9 : 1.0);
    chk(beta, -31.0);
    double alpha = 2.0 - det_pow<false>(beta,-31.0);
    chk(r*alpha, 1.0/31.0);
    chk(1.0/(2.0 - r*alpha), 1.0/31.0);
    // PM: xy in [0,1], y = 21 ; val in (0,2], y = 1/21
    double xy = U(g) < 0.2 ? std::pow(2.0, -60.0*U(g)) : U(g);
    chk(xy, 21.0);
    chk(2.0*r + (1.0-2.0*r)*det_pow<false>(xy,21.0), 1.0/21.0);
    chk(std::ldexp(U(g), -(int)(40*U(g))), 21.0);
  }
  printf("checked %ld, mismatches %ld\n", n, bad);
  return bad != 0;
}
