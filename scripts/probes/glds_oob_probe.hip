// Probe: does a range-checked (out-of-bounds) buffer_load ... lds write ZEROS into LDS, or leave
// the destination untouched? The implicit-GEMM convolution's zero padding relies on the answer.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void k(const uint32_t* g, uint32_t bytes, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) lds[i] = 0xABABABABu;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(g), (short)0,
                                                               (int)bytes, 0x00020000);
  const uint32_t voff = (threadIdx.x & 1) ? 0x80000000u : threadIdx.x * 16u;
  typedef __attribute__((address_space(3))) void* lptr;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lptr)(lds + (threadIdx.x / 64) * 256), 16, voff, 0, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) out[i] = lds[i];
}

int main() {
  uint32_t h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = 0x1000 + i;
  uint32_t *g, *o;
  hipMalloc(&g, sizeof(h));
  hipMalloc(&o, sizeof(h));
  hipMemcpy(g, h, sizeof(h), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, g, (uint32_t)sizeof(h), o);
  uint32_t r[1024];
  hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
  int in_ok = 0, oob_zero = 0, oob_kept = 0, other = 0;
  for (int t = 0; t < 256; ++t)
    for (int j = 0; j < 4; ++j) {
      const uint32_t v = r[t * 4 + j];
      if (t & 1) { if (v == 0) ++oob_zero; else if (v == 0xABABABABu) ++oob_kept; else ++other; }
      else { if (v == h[t * 4 + j]) ++in_ok; else ++other; }
    }
  printf("in-bounds correct %d/512, oob->zero %d, oob->untouched %d, other %d\n", in_ok, oob_zero,
         oob_kept, other);
  return 0;
}
