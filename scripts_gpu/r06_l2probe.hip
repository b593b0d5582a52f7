// r06 probe: is data written by one kernel seen by every XCD in the next kernel of the same
// stream, when the reading XCDs still hold copies of the old lines from an earlier kernel?
//   read_all  : every workgroup reads the whole buffer P (each XCD's L2 now holds P's lines)
//   write_some: a few workgroups overwrite P with the iteration's value (plain stores)
//   check_all : every workgroup reads P again and counts words != the new value
// Counts stale words per iteration over many iterations, for several buffer sizes, with and
// without an eviction kernel between the first read and the write. Build:
//   hipcc --offload-arch=gfx950 -O2 -o scripts_gpu/r06_l2probe scripts_gpu/r06_l2probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void read_all(const float* p, int n, float* sink) {
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += p[i];
  if (s == 12345.f) sink[blockIdx.x] = s;  // keep the loads
}

__global__ void write_some(float* p, int n, float v) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = v;
}

__global__ void check_all(const float* p, int n, float v, unsigned* bad) {
  unsigned c = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) c += p[i] != v;
  if (c) atomicAdd(bad, c);
}

__global__ void evict(const float4* q, long n, float* sink) {
  float s = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) s += q[i].x;
  if (s == 12345.f) sink[0] = s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  float *p, *sink, *ev;
  unsigned* bad;
  const int nmax = 1 << 20;
  const long evn = 64L << 20;  // 1 GiB of float4
  CK(hipMalloc(&p, nmax * sizeof(float)));
  CK(hipMalloc(&sink, 4096 * sizeof(float)));
  CK(hipMalloc(&bad, sizeof(unsigned)));
  CK(hipMalloc(&ev, evn * 16));
  CK(hipMemset(ev, 0, evn * 16));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int sizes[] = {1024, 16384, 262144};
  for (int ev_on = 0; ev_on < 2; ++ev_on) {
    for (int n : sizes) {
      for (int wg : {1, 8, 64}) {
        CK(hipMemsetAsync(p, 0, n * sizeof(float), s));
        unsigned tot = 0, hit = 0;
        for (int it = 1; it <= iters; ++it) {
          CK(hipMemsetAsync(bad, 0, sizeof(unsigned), s));
          hipLaunchKernelGGL(read_all, dim3(1024), dim3(256), 0, s, p, n, sink);
          if (ev_on) hipLaunchKernelGGL(evict, dim3(4096), dim3(256), 0, s, (const float4*)ev, evn, sink);
          hipLaunchKernelGGL(write_some, dim3(wg), dim3(256), 0, s, p, n, (float)it);
          hipLaunchKernelGGL(check_all, dim3(1024), dim3(256), 0, s, p, n, (float)it, bad);
          unsigned b = 0;
          CK(hipMemcpyAsync(&b, bad, sizeof(unsigned), hipMemcpyDeviceToHost, s));
          CK(hipStreamSynchronize(s));
          tot += b;
          hit += b != 0;
        }
        printf("evict=%d n=%7d words, writer wgs=%2d: %u of %d iterations saw stale words (%u stale word reads)\n", ev_on,
               n, wg, hit, iters, tot);
        fflush(stdout);
      }
    }
  }
  CK(hipFree(p));
  CK(hipFree(ev));
  return 0;
}
