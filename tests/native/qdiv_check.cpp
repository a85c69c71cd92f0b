// Exhaustive-style check of kg_qdiv (kg_common.h): the fp32-estimate + one-correction quotient
// must equal Go/C int64 division on every operand it takes the fast path for, including the
// boundaries n = k·d and n = k·d ± 1.  Built and run by tests/test_qdiv_cpu.py.
#include "kg_common.h"
#include <cstdlib>
#include <random>
#include <cstdio>
int main(int argc, char **argv){ std::mt19937_64 g(1); long bad=0, n_=0;
 const long iters = argc > 1 ? atol(argv[1]) : 2000000;
 for(long it=0;it<iters;it++){ int64_t d = (g()% (1LL<< (1+g()%40))) + 1; if(d>=(1LL<<40)) d=(1LL<<40)-1;
   int64_t k = g()%129; int64_t n; int mode=g()%4;
   if(mode==0) n=k*d; else if(mode==1) n=k*d-1; else if(mode==2) n=k*d+1; else n=(int64_t)(g()% (uint64_t)(128*d));
   if(n<0) n=0; n_++; if(kg_qdiv(n,d)!=n/d){ if(bad<5) printf("bad n=%ld d=%ld got %ld want %ld\n",n,d,kg_qdiv(n,d),n/d); bad++;} }
 printf("checked %ld bad %ld\n",n_,bad); return bad != 0; }
