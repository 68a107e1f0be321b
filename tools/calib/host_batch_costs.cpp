// Host-side bookkeeping of a 1M-packet parseBatch, without the GPU: shared_ptr copies of each
// packet's data (the batch keeps its frames alive), a fresh 96-MB record array faulted in by T
// threads, its free, and the serial release of the references. Build: g++ -O2 -std=c++17 -pthread
#include <memory>
#include <vector>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <cstdlib>
using C = std::chrono::steady_clock;
double ms(C::time_point a, C::time_point b){return std::chrono::duration<double,std::milli>(b-a).count();}
int main(int argc, char** argv){
  const size_t n=1<<20;
  std::vector<std::shared_ptr<const uint8_t[]>> pk(n);
  for(size_t i=0;i<n;++i){ pk[i]=std::shared_ptr<const uint8_t[]>(new uint8_t[64]); }
  for(int rep=0;rep<3;++rep){
    auto t0=C::now();
    std::vector<std::shared_ptr<const uint8_t[]>> keep(n);
    int T=argc > 1 ? atoi(argv[1]) : 16; std::vector<std::thread> th;
    for(int w=0;w<T;++w) th.emplace_back([&,w]{ for(size_t i=n*w/T;i<n*(w+1)/T;++i) keep[i]=pk[i]; });
    for(auto&x:th) x.join();
    auto t1=C::now();
    std::vector<uint8_t> recs; recs.reserve(n*96); 
    struct R{uint8_t b[96];};
    R* r = static_cast<R*>(::operator new(n*96));
    std::vector<uint8_t> src(n*96/16, 1);
    th.clear();
    for(int w=0;w<T;++w) th.emplace_back([&,w]{ for(size_t i=n*w/T;i<n*(w+1)/T;i+=1) std::memcpy(&r[i], src.data()+(i%1000)*96, 96); });
    for(auto&x:th) x.join();
    auto t2=C::now();
    ::operator delete(r);
    auto t3=C::now();
    keep.clear(); keep.shrink_to_fit();
    auto t4=C::now();
    printf("keep copy %.2f ms, recs fault+fill %.2f ms, free %.2f ms, keep release %.2f ms\n", ms(t0,t1), ms(t1,t2), ms(t2,t3), ms(t3,t4));
  }
}
