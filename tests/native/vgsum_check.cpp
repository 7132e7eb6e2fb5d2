// vgsum_check.cpp — replays libstdc++'s introsort levels over key
// arrays dumped by the oracle (LEGO_ORACLE_VG_DUMP: int32 count, then the
// keys, per VoxelGrid call) and checks lego_vgsort.h's sumOrder rule: with the
// heap pieces it ranks stably (each key at most twice in the piece, the
// smallest not also in the preceding leaf) and the others heap-sorted, every
// voxel's float sum from 0 of random values equals the sum in std::sort's
// order.  tests/test_numerics_shim.py::test_vgsort_sum_order_rule runs it
// over the C2 ring keys and adversary fixtures; by hand: g++ -O2 -std=c++17
// tests/native/vgsum_check.cpp -o /tmp/vgsum && /tmp/vgsum dump.bin (V=1
// lists the ranked pieces).  Exit status 1 when a voxel sum differs.
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>
#include <cstring>
using namespace std;
struct E { unsigned k; int v; };
static void med(vector<E>& a,int r,int x,int y,int z){ int m; if(a[x].k<a[y].k){ if(a[y].k<a[z].k) m=y; else if(a[x].k<a[z].k) m=z; else m=x;} else if(a[x].k<a[z].k) m=x; else if(a[y].k<a[z].k) m=z; else m=y; swap(a[r],a[m]);}
static int part(vector<E>& a,int f,int l){ int mid=f+(l-f)/2; med(a,f,f+1,mid,l-1); int p=f; int i=f+1,j=l; while(true){ while(a[i].k<a[p].k) ++i; --j; while(a[p].k<a[j].k) --j; if(!(i<j)) return i; swap(a[i],a[j]); ++i;} }
struct Piece{int s,e; bool heap;};
static void rec(vector<E>& a,int f,int l,int depth,vector<Piece>& P){
  if(l-f<=16){ if(l>f) P.push_back({f,l,false}); return; }
  if(depth==0){ P.push_back({f,l,true}); return; }
  int c=part(a,f,l); rec(a,f,c,depth-1,P); rec(a,c,l,depth-1,P);
}
int main(int argc,char**argv){ FILE* f=fopen(argv[1],"rb"); int m; int call=0; int bad=0, shortcuts=0, flagged=0;
 mt19937 rng(1);
 while(fread(&m,4,1,f)==1){ vector<unsigned> keys(m); if(fread(keys.data(),4,m,f)!=(size_t)m) return 1; call++;
   vector<E> ref(m); for(int i=0;i<m;i++) ref[i]={keys[i],i};
   vector<E> a=ref; sort(ref.begin(),ref.end(),[](const E&x,const E&y){return x.k<y.k;});
   vector<Piece> P; int D=m>1?2*(31-__builtin_clz(m)):0; rec(a,0,m,D,P);
   vector<E> out(m);
   for(size_t pi=0;pi<P.size();pi++){ auto pc=P[pi]; vector<E> seg(a.begin()+pc.s,a.begin()+pc.e);
     bool exact=!pc.heap;
     if(pc.heap){ // rule
       bool ex=false; unsigned mn=~0u; for(auto&e:seg) mn=min(mn,e.k);
       for(auto&e:seg){ int c=0; for(auto&g:seg) c+=g.k==e.k; if(c>=3) ex=true; if(c==2 && e.k==mn && pi>0){ auto pp=P[pi-1]; for(int q=pp.s;q<pp.e;q++) if(a[q].k==mn) ex=true; } }
       exact=ex; if(ex) flagged++; else { shortcuts++; if(getenv("V")) printf("call %d n=%d shortcut piece [%d,%d)\n",call,m,pc.s,pc.e);} 
     }
     if(pc.heap && exact){ make_heap(seg.begin(),seg.end(),[](const E&x,const E&y){return x.k<y.k;}); sort_heap(seg.begin(),seg.end(),[](const E&x,const E&y){return x.k<y.k;}); }
     else stable_sort(seg.begin(),seg.end(),[](const E&x,const E&y){return x.k<y.k;});
     copy(seg.begin(),seg.end(),out.begin()+pc.s);
   }
   // random point values: compare voxel sums
   vector<float> val(m); uniform_real_distribution<float> U(-10,10); for(auto&x:val) x=U(rng);
   for(int i=0;i<m;){ int j=i; float s1=0,s2=0; while(j<m && ref[j].k==ref[i].k){ s1+=val[ref[j].v]; s2+=val[out[j].v]; if(out[j].k!=ref[j].k){bad++; break;} j++; } if(memcmp(&s1,&s2,4)) { bad++; printf("call %d voxel at %d differs\n",call,i);} i=j; }
 }
 printf("calls %d shortcuts %d flagged %d bad %d\n",call,shortcuts,flagged,bad);
 return bad ? 1 : 0;
}
