/* cdc_edge.c -- one more CDC hypothesis family (round 2): the zpaq recurrence
 * with its state reset at READ-BUFFER edges (a chunker whose find_boundary
 * keeps state in locals), buffers of 100 B .. 64 KiB, h and/or o1 reset,
 * both multiplier orders, every predicate width, both cut sides.  Prints the
 * variants whose first cut is the KAT's 11,579 (src/index.rs:771): none.
 * Research tool only.  gcc -O2 -o /tmp/cdc_edge scripts/cdc_edge.c && /tmp/cdc_edge */
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static uint8_t buf[64<<10]; static int n;
int main(void){
  n=0; for(int i=1;i<=2000;++i) n+=sprintf((char*)buf+n,"Line %d\n",i);
  for(int i=0;i<2000;++i) n+=sprintf((char*)buf+n,"Test content\n");
  const uint32_t MP[2][2]={{314159265u,271828182u},{271828182u,314159265u}};
  int bsizes[64]; int nb=0;
  for(int b=256;b<=65536;b*=2) bsizes[nb++]=b;
  int extra[]={1000,3000,5000,6000,10000,12000,4000,8000,16000,32000,100,500,1500,2500,7000,9000,11000,11579,11578};
  for(unsigned i=0;i<sizeof extra/sizeof *extra;i++) bsizes[nb++]=extra[i];
  long found=0;
  for(int bi=0;bi<nb;bi++) for(int mp=0;mp<2;mp++) for(int rs=1;rs<4;rs++) for(int refeed=0;refeed<2;refeed++)
  for(int k=1;k<=31;k++) for(int incl=0;incl<2;incl++){
    int B=bsizes[bi];
    uint32_t h=0; uint8_t c1=0, o1[256]; memset(o1,0,256);
    int first=-1;
    // process in buffers of B bytes; at each buffer start apply reset policy rs (1: h, 2: o1/c1, 3: both)
    // refeed: buffer start positions are multiples of B from 0, but each call re-feeds from the
    // chunk start within the buffer (only matters after cuts; first chunk: same as no refeed)
    for(int start=0; start<n && first<0; start+=B){
      if(start>0){ if(rs&1) h=0; if(rs&2){ c1=0; memset(o1,0,256);} }
      int end=start+B<n?start+B:n;
      for(int i=start;i<end;i++){
        uint8_t c=buf[i];
        uint32_t M = (c==o1[c1])?MP[mp][0]:MP[mp][1];
        h=(h+c+1u)*M; o1[c1]=c; c1=c;
        if(h < (1u<<k)){ first = incl? i+1 : i; break; }
      }
    }
    if(first==11579){ found++; printf("B=%d mp=%d rs=%d k=%d incl=%d\n",B,mp,rs,k,incl);}
  }
  printf("found %ld\n",found);
}
