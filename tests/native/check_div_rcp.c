/* Exhaustive check of librsd's div_rcp (csrc/svao_math.h) against IEEE binary32 division:
 * for every divisor b given on the command line, every numerator a = 0 or a in [2^-60, 2^31]
 * (div_rcp's precondition) must give the bits of a / b.  Used by tests/test_div_rcp.py; the
 * arithmetic is the same five FMA/MUL steps the kernels execute.  Optional env LIMIT_BINADES
 * restricts the numerators to that many binades from 2^-60, or from 2^START_EXP (quick CPU test). */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>
static float fb(uint32_t u){float f;memcpy(&f,&u,4);return f;}
static uint32_t bf(float f){uint32_t u;memcpy(&u,&f,4);return u;}
static float div_rcp(float a,float b,float y){float q0=a*y;float r0=fmaf(-q0,b,a);float q1=fmaf(r0,y,q0);float r1=fmaf(-q1,b,a);return fmaf(r1,y,q1);}
typedef struct {float b; uint32_t lo,hi; uint64_t bad;} job;
static void* run(void* p){job*j=p;float y=(float)(1.0/(double)j->b);for(uint32_t u=j->lo;u<j->hi;u++){float a=fb(u);float q=a/j->b;float r=div_rcp(a,j->b,y);if(bf(q)!=bf(r)){if(j->bad<3)printf("MISMATCH b=%a a=%a q=%a r=%a\n",j->b,a,q,r);j->bad++;}}return 0;}
int main(int argc,char**argv){
  // numerators: 0 and all floats in [2^-60, 2^31]
  uint32_t lo=bf(0x1p-60f), hi=bf(0x1p31f)+1;
  const char* st=getenv("START_EXP"); if(st) lo=bf(ldexpf(1.0f,atoi(st)));
  const char* lb=getenv("LIMIT_BINADES"); if(lb){int k=atoi(lb); uint32_t h2=lo+((uint32_t)k<<23); if(h2<hi) hi=h2;}
  int nb=argc-1; uint64_t tot=0;
  for(int k=0;k<nb;k++){float b=strtof(argv[k+1],0); job J[8]; pthread_t t[8]; uint32_t n=hi-lo;
    for(int i=0;i<8;i++){J[i].b=b;J[i].lo=lo+(uint64_t)n*i/8;J[i].hi=lo+(uint64_t)n*(i+1)/8;J[i].bad=0;pthread_create(&t[i],0,run,&J[i]);}
    uint64_t bad=0; for(int i=0;i<8;i++){pthread_join(t[i],0);bad+=J[i].bad;}
    float y=(float)(1.0/(double)b); float z=div_rcp(0.0f,b,y); if(bf(z)!=bf(0.0f/b)) bad++;
    printf("b=%a bad=%llu\n",b,(unsigned long long)bad); tot+=bad;}
  printf("total bad %llu\n",(unsigned long long)tot); return 0;}
