// Simulate "speculative cascades": per batch (bucket L snapshot), items popped in FIFO order;
// an interrupting item's cascade (levels < L) runs to exhaustion right after it. Batch is cut
// at the first event whose read set intersects the write set of an EARLIER cascade in this batch.
#include <stdint.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>
static int H,W; static const uint8_t*IMG; static int32_t*M;
static int cd(int p,int q){const uint8_t*a=IMG+3*p,*b=IMG+3*q;int d0=abs(a[0]-b[0]),d1=abs(a[1]-b[1]),d2=abs(a[2]-b[2]);int m=d0>d1?d0:d1;return m>d2?m:d2;}
typedef struct{int32_t*v;size_t h,n,c;}Q; static Q q[256];
static void push(Q*q,int32_t x){if(q->n==q->c){q->c=q->c?q->c*2:1024;q->v=realloc(q->v,q->c*4);}q->v[q->n++]=x;}
static int32_t*wstamp; // batch id + cascade rank that wrote the pixel (0 = none this batch)
static long long cur_batch=0;
// stamp encoding: (batch<<24)|(c+1) but c can exceed 2^24 -> use two arrays
static int64_t*wb; static int32_t*wc;
static int conflict_read(int p,int rank){ // does p's state come from an earlier cascade (rank'<rank)?
  return wb[p]==cur_batch && wc[p]<rank; }
static int readset_conflict(int p,int rank){ int nb[4]={p-1,p+1,p-W,p+W};
  if(conflict_read(p,rank))return 1;
  for(int k=0;k<4;k++){ if(conflict_read(nb[k],rank))return 1; }
  return 0;}
static void wr(int p,int rank){wb[p]=cur_batch;wc[p]=rank;}
// pop one pixel serially; returns mask of low pushes in *low; records writes with rank 'rank' if rank>=0
static int pop(int p,int L,int rank,int*lowlist,int*nlow){int nb[4]={p-1,p+1,p-W,p+W};int lab=0;
  for(int k=0;k<4;k++){int t=M[nb[k]];if(t>0){if(!lab)lab=t;else if(t!=lab)lab=-1;}}
  M[p]=lab; if(rank>=0)wr(p,rank); if(lab==-1)return 0; int any=0;
  for(int k=0;k<4;k++)if(M[nb[k]]==0){int t=cd(p,nb[k]);M[nb[k]]=-2;if(rank>=0)wr(nb[k],rank);
     if(t<L){lowlist[(*nlow)++]=nb[k];lowlist[H*W+8+(*nlow)-1]=t;any=1;} else push(&q[t],nb[k]);}
  return any;}
int main(int argc,char**argv){H=atoi(argv[1]);W=atoi(argv[2]);int BUDGET=argc>3?atoi(argv[3]):1000000;
 uint8_t*img=malloc((size_t)H*W*3);M=malloc((size_t)H*W*4);if(fread(img,1,(size_t)H*W*3,stdin)){};if(fread(M,4,(size_t)H*W,stdin)){};IMG=img;
 wb=calloc((size_t)H*W,8);wc=calloc((size_t)H*W,4);
 for(int c=0;c<W;c++){M[c]=-1;M[(H-1)*W+c]=-1;}
 for(int r=1;r<H-1;r++){M[r*W]=-1;M[r*W+W-1]=-1;for(int c=1;c<W-1;c++){int p=r*W+c;if(M[p]<0)M[p]=0;if(M[p])continue;int l=256;
   int nb[4]={p-1,p+1,p-W,p+W};for(int k=0;k<4;k++)if(M[nb[k]]>0){int t=cd(p,nb[k]);if(t<l)l=t;}
   if(l<256){push(&q[l],p);M[p]=-2;}}}
 long long iters=0,cas=0,maxcas=0,sumcasmax=0; int*low=malloc(sizeof(int)*2*((size_t)H*W+8)); 
 // local cascade queue: simple per-level FIFOs
 Q lq[256];memset(lq,0,sizeof lq);
 for(;;){int L=0;while(L<256&&q[L].h==q[L].n)L++;if(L==256)break; iters++; cur_batch=iters;
   size_t end=q[L].n; int rank=0; long long batchmaxcas=0;
   while(q[L].h<end){int p=q[L].v[q[L].h]; rank++;
     if(readset_conflict(p,rank)) break;      // cut before this item (stays queued)
     q[L].h++; int nlow=0; int any=pop(p,L,-1,low,&nlow);
     if(!any) continue;
     // cascade: serial flood at levels < L from the low pushes, rank = 'rank' (after item)
     for(int k=0;k<nlow;k++){int t=low[H*W+8+k]; push(&lq[t],low[k]); wr(low[k],rank);} 
     long long len=0; int conflict=0; 
     for(;;){int a=0;while(a<L&&lq[a].h==lq[a].n)a++; if(a>=L)break; int x=lq[a].v[lq[a].h++]; len++;
        if(readset_conflict(x,rank)) conflict=1;
        int nl=0; pop(x,L,rank,low,&nl); for(int k=0;k<nl;k++){int t=low[H*W+8+k];push(&lq[t],low[k]);} }
     for(int a=0;a<L;a++){lq[a].h=lq[a].n=0;}
     cas++; if(len>maxcas)maxcas=len; if(len>batchmaxcas)batchmaxcas=len;
     if(conflict||len>BUDGET){ /* in the real engine: cut after x (cascade redone as normal batches) */ 
        // the simulation already applied it serially; count an extra iteration per conflict
        iters++; break; }
   }
   sumcasmax+=batchmaxcas;
 }
 printf("%dx%d iters=%lld cascades=%lld maxcascade=%lld sum(batch max cascade)=%lld px/iter=%.1f\n",H,W,iters,cas,maxcas,sumcasmax,(double)H*W/iters);}
