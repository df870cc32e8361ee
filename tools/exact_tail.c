// structured exact search for next(h0u,h0,h0d,h1u,h1,h1d,a) with
// 2 symmetric LUT3 over A + 2 symmetric LUT3 over B + a 3-LUT tail over {gA1,gA2,gB1,gB2,a}
#include <stdio.h>
#include <stdint.h>
static uint32_t lut(uint32_t tt, uint32_t x, uint32_t y, uint32_t z){
  uint32_t r=0; for(int k=0;k<8;k++) if(tt>>k&1){ uint32_t m=((k&4)?x:~x)&((k&2)?y:~y)&((k&1)?z:~z); r|=m;} return r;}
static int dep(uint32_t F, uint32_t x, uint32_t y, uint32_t z){
  for(int k=0;k<8;k++){ uint32_t m=((k&4)?x:~x)&((k&2)?y:~y)&((k&1)?z:~z); if((m&F)&&(m&~F)) return 0;} return 1;}
int main(){
  // domain: (SA in 0..3, SB in 0..3, a in 0,1) with a consistent with ... a is the centre which is in h0/h1 -- treat as free (superset)
  // use 32 minterms: SA(2b) SB(2b) a(1b)
  long cand=0, total=0;
  for(int fa1=0;fa1<16;fa1++)for(int fa2=fa1+1;fa2<16;fa2++)
  for(int fb1=0;fb1<16;fb1++)for(int fb2=fb1+1;fb2<16;fb2++){
    uint32_t s[5]={0},F=0;
    for(int m=0;m<32;m++){int SA=m&3,SB=m>>2&3,a=m>>4&1; int c=SA+2*SB;
      if(fa1>>SA&1) s[0]|=1u<<m; if(fa2>>SA&1) s[1]|=1u<<m; if(fb1>>SB&1) s[2]|=1u<<m; if(fb2>>SB&1) s[3]|=1u<<m; if(a) s[4]|=1u<<m;
      if(c==3||(a&&c==4)) F|=1u<<m;}
    // F must be a function of s[0..4]
    int ok=1; for(int m=0;m<32&&ok;m++)for(int n=m+1;n<32;n++){int same=1;for(int i=0;i<5;i++) if(((s[i]>>m)^(s[i]>>n))&1){same=0;break;} if(same&&(((F>>m)^(F>>n))&1)){ok=0;break;}}
    if(!ok) continue; cand++;
    uint32_t sig[7]; for(int i=0;i<5;i++) sig[i]=s[i];
    for(int a1=0;a1<5;a1++)for(int b1=a1+1;b1<5;b1++)for(int c1=b1+1;c1<5;c1++)
    for(int t1=0;t1<256;t1++){ sig[5]=lut(t1,sig[a1],sig[b1],sig[c1]);
     for(int a3=0;a3<6;a3++)for(int b3=a3+1;b3<6;b3++) if(dep(F,sig[a3],sig[b3],sig[5])){printf("2-gate tail fa=%x,%x fb=%x,%x\n",fa1,fa2,fb1,fb2);}
     for(int a2=0;a2<6;a2++)for(int b2=a2+1;b2<6;b2++)for(int c2=b2+1;c2<6;c2++)
     for(int t2=0;t2<256;t2++){ sig[6]=lut(t2,sig[a2],sig[b2],sig[c2]);
      for(int a3=0;a3<6;a3++)for(int b3=a3+1;b3<6;b3++) if(dep(F,sig[a3],sig[b3],sig[6])){
        total++; if(total<20) printf("fa=%x,%x fb=%x,%x g1=(%d,%d,%d)%02x g2=(%d,%d,%d)%02x g3=(%d,%d,g2)\n",fa1,fa2,fb1,fb2,a1,b1,c1,t1,a2,b2,c2,t2,a3,b3);}
     }}
  }
  printf("cand %ld total %ld\n",cand,total);
}
