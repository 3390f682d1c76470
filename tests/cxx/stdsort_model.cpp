// stdsort_model.cpp — CPU check of the formulation behind vloam-noted_amd/csrc/stdsort.h.
//
// The device reproduces libstdc++'s std::sort permutation (key-only comparator, the sort of
// scan_registration.cpp:365-366 and of PCL VoxelGrid) with a parallel restatement of the Hoare
// scan (stop lists, swap count S, cut = min(l_{S+1}, r_S)), segments processed in any order,
// the depth-limit heap sort and a per-segment stable final pass.  This program runs the same
// formulation serially (segments popped in random order) and compares it with std::sort itself
// on 20k random inputs (heavy ties, sorted, reversed, tiny) and median-of-3-adversarial
// patterns that reach the heap-sort fallback.  Exit status 0 iff every permutation matches and
// the heap path was exercised.  Built and run by tests/test_host_models.py.
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>
typedef uint64_t T;
static bool less_(T a, T b){ return (uint32_t)(a>>32) < (uint32_t)(b>>32); }
static void adjust(std::vector<T>&E,int first,int hole,int len,T value){
  int top=hole, second=hole;
  while(second < (len-1)/2){ second=2*(second+1); if(less_(E[first+second],E[first+second-1])) second--; E[first+hole]=E[first+second]; hole=second; }
  if((len&1)==0 && second==(len-2)/2){ second=2*(second+1); E[first+hole]=E[first+second-1]; hole=second-1; }
  int parent=(hole-1)/2;
  while(hole>top && less_(E[first+parent],value)){ E[first+hole]=E[first+parent]; hole=parent; parent=(hole-1)/2; }
  E[first+hole]=value;
}
static long heaps=0; static void heapsort(std::vector<T>&E,int lo,int hi){ heaps++;
  int len=hi-lo; if(len>=2){ int parent=(len-2)/2; while(true){ T v=E[lo+parent]; adjust(E,lo,parent,len,v); if(parent==0)break; parent--; } }
  int last=hi; while(last-lo>1){ --last; T v=E[last]; E[last]=E[lo]; adjust(E,lo,0,last-lo,v);} }
static std::vector<T> emul(std::vector<T> E){
  int n=E.size(); std::vector<uint32_t> A(n+1),B(n+1);
  struct Seg{int lo,hi,d;}; std::vector<Seg> st;
  if(n>16) st.push_back({0,n,2*(31-__builtin_clz(n))});
  auto mark=[&](int lo,int hi,bool sorted){ for(int i=lo;i<hi;i++){A[i]=sorted?i:lo;B[i]=sorted?i+1:hi;} };
  // random processing order to check order-independence
  std::mt19937 g(5);
  while(!st.empty()){
    int pick=g()%st.size(); Seg s=st[pick]; st.erase(st.begin()+pick);
    int lo=s.lo,hi=s.hi,d=s.d;
    while(true){
      if(hi-lo<=16){ mark(lo,hi,false); break; }
      if(d==0){ heapsort(E,lo,hi); mark(lo,hi,true); break; }
      --d;
      int a=lo+1,b=lo+(hi-lo)/2,c=hi-1,m;
      if(less_(E[a],E[b])){ if(less_(E[b],E[c])) m=b; else if(less_(E[a],E[c])) m=c; else m=a; }
      else if(less_(E[a],E[c])) m=a; else if(less_(E[b],E[c])) m=c; else m=b;
      std::swap(E[lo],E[m]); T p=E[lo];
      int nl=0,nr=1; B[lo]=lo;
      for(int i=lo+1;i<hi;i++){ if(!less_(E[i],p)) A[lo+1+nl++]=i; if(!less_(p,E[i])) B[lo+nr++]=i; }
      int kmax=std::min(nl,nr),S=0; for(int k=1;k<=kmax;k++){ if(A[lo+k]<B[lo+nr-k]) S++; else break; }
      int lK= S+1<=nl? (int)A[lo+S+1]:0x7fffffff; int rS= S>=1? (int)B[lo+nr-S]:hi; int cut=std::min(lK,rS);
      for(int k=1;k<=S;k++) std::swap(E[A[lo+k]],E[B[lo+nr-k]]);
      if(hi-cut>16) st.push_back({cut,hi,d}); else mark(cut,hi,false);
      hi=cut;
    }
  }
  std::vector<T> out(n);
  for(int i=0;i<n;i++){ int lo,hi; if(n<=16){lo=0;hi=n;} else {lo=A[i];hi=B[i];} int r=0; for(int j=lo;j<hi;j++) r+= (less_(E[j],E[i]) || (j<i && !less_(E[i],E[j]))); out[lo+r]=E[i]; }
  return out;
}
int main(){
  std::mt19937_64 g(1); long bad=0, tot=0;
  for(int it=0;it<20000;it++){
    int n = (it%7==0)? g()%20 : 1+g()%3000; int kv = 1+g()% (it%3==0? 4 : (it%3==1? 50 : 100000));
    std::vector<T> v(n); for(int i=0;i<n;i++) v[i]=((T)(g()%kv)<<32)|i;
    if(it%11==0) std::sort(v.begin(),v.end(),[](T a,T b){return a<b;}); // sorted input
    if(it%13==0) std::reverse(v.begin(),v.end());
    auto r=v; std::sort(r.begin(),r.end(),less_);
    auto e=emul(v); tot++; if(e!=r){ bad++; if(bad<5) printf("mismatch n=%d kv=%d\n",n,kv);} }
  // median-of-3 killer style: organ pipe + sawtooth patterns forcing depth limit
  for(int n: {100,500,1000,2049,4096}){ for(int pat=0;pat<4;pat++){
    std::vector<T> v(n); for(int i=0;i<n;i++){ uint32_t k; if(pat==0) k=(i%2)? i: n-i; else if(pat==1) k= i<n/2? i: n-i; else if(pat==2) k=(i*7919)%n / 3; else k = (i & 1) ? i/2 : n - i/2; v[i]=((T)k<<32)|i; }
    // classic median-of-3 killer (Musser)
    if(pat==3){ int k=n/2; for(int i=0;i<k;i++){ uint32_t a = (i%2==0)? i+1 : k+i; v[i]=((T)a<<32)|i; } for(int i=k;i<n;i++){ v[i]=((T)(2*(i-k+1))<<32)|i; } }
    auto r=v; std::sort(r.begin(),r.end(),less_); auto e=emul(v); tot++; if(e!=r){bad++; printf("adv mismatch n=%d pat=%d\n",n,pat);} } }
  printf("cases %ld mismatches %ld heap sorts %ld\n",tot,bad,heaps); return (bad!=0 || heaps==0); }
