// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DQP_STAMPS -I sdf-nmpc_amd/csrc tools/qp_stamps_drv.hip sdf-nmpc_amd/csrc/rti_qp.hip -o tools/_qp_stamps_drv
// standalone diagnostic driver: synthetic QP inputs from files written by tools/qp_stamps.py
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "qp_kernels.h"
using namespace sdfn;
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb"); int B, N; fread(&B, 4, 1, f); fread(&N, 4, 1, f);
  const char* names[] = {"xn","AB","y","Jy","yN","JyN","h","Jh","x","u","x0","yref","W","yNref","WN","dt"};
  size_t sizes[] = {(size_t)B*N*10,(size_t)B*N*140,(size_t)B*N*11,(size_t)B*N*154,(size_t)B*4,(size_t)B*40,(size_t)B*(N+1)*3,(size_t)B*(N+1)*30,(size_t)B*(N+1)*10,(size_t)B*N*4,(size_t)B*10,(size_t)B*N*11,(size_t)B*N*11,(size_t)B*4,(size_t)B*4,(size_t)N};
  double* d[16];
  for (int i=0;i<16;++i){ std::vector<double> h(sizes[i]); fread(h.data(),8,sizes[i],f); hipMalloc(&d[i],8*sizes[i]); hipMemcpy(d[i],h.data(),8*sizes[i],hipMemcpyHostToDevice);} 
  double opt[22]; fread(opt, 8, 22, f); fclose(f);
  QpArgs q{}; q.B=B; q.N=N; q.xn=d[0];q.AB=d[1];q.y=d[2];q.Jy=d[3];q.yN=d[4];q.JyN=d[5];q.h=d[6];q.Jh=d[7];q.x=d[8];q.u=d[9];q.x0=d[10];q.yref=d[11];q.W=d[12];q.yNref=d[13];q.WN=d[14];q.dt=d[15];
  for(int i=0;i<4;++i){q.lbu[i]=opt[i];q.ubu[i]=opt[4+i];} for(int i=0;i<3;++i){q.lh[i]=opt[8+i];q.uh[i]=opt[11+i];q.zl[i]=opt[14+i];q.Zl[i]=opt[17+i];} qp_default_rows(q);
  q.lm=opt[20]; q.tol=opt[21]; q.max_iter=100; q.cost_scaling=1; q.lm_scaling=1; q.ny=11;
  hipMalloc(&q.dx,8*B*(N+1)*10); hipMalloc(&q.du,8*B*N*4); hipMalloc(&q.status,4*B); hipMalloc(&q.iters,4*B); hipMalloc(&q.res,16*B);
  hipMalloc(&q.work,8*B*qp_work_doubles(N)); hipMalloc(&q.stamps,8*B*16);
  for (int r=0;r<3;++r) { launch_rti_qp_pack(q,0); launch_rti_qp(q,0); }
  hipEvent_t a,b; hipEventCreate(&a); hipEventCreate(&b); launch_rti_qp_pack(q,0); hipEventRecord(a); launch_rti_qp(q,0); hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms,a,b);
  std::vector<double> st(B*16); hipMemcpy(st.data(),q.stamps,8*B*16,hipMemcpyDeviceToHost);
  std::vector<int> it(B); hipMemcpy(it.data(),q.iters,4*B,hipMemcpyDeviceToHost);
  double tot[16]={0}; int mx=0; for(int i=0;i<B;++i){for(int j=0;j<16;++j) tot[j]+=st[i*16+j]; if(it[i]>mx)mx=it[i];}
  const char* ph[]={"setup","sweep0","bwd-factor","fwd(x2)","rows-pred+terms","bwd-corr","rows-upd+terms","c:pos+entry","8:f-entry+W|r-pred","9:f-M_u|r-update","f:chol+kg","f:jos->Pa","f:stores","c:reads","c:chain","c:tail"};
  double mi=0; for(int i=0;i<B;++i) mi+=it[i]; std::vector<int> stt(B); hipMemcpy(stt.data(),q.status,4*B,hipMemcpyDeviceToHost); int nc=0; for(int i=0;i<B;++i) nc+=stt[i]!=0;
  printf("kernel %.3f ms, max iters %d, mean %.2f, not converged %d\n", ms, mx, mi/B, nc); double s=0; for(int j=0;j<16;++j) s+=tot[j];
  for(int j=0;j<16;++j) printf("  %-14s %8.0f cycles/instance (%.1f%%)\n", ph[j], tot[j]/B, 100*tot[j]/s);
  return 0; }
