// Repro for the C4 rocprofv3 --pmc teardown SIGSEGV:
// does a process that made ONE hipLaunchCooperativeKernel call crash in exit()
// after rocprofv3's tool finalization, with none of libaaa.so loaded?
//   coop_exit coop        one cooperative launch of a trivial 256-WG kernel
//   coop_exit plain       the same kernel, ordinary launch
//   coop_exit coop_sync   cooperative launch, then hipDeviceSynchronize + hipStreamDestroy of nothing
// Run under: rocprofv3 --pmc SQ_WAVES -- ./coop_exit <mode>; compare exit codes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__global__ void k_touch(int* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = (int)blockIdx.x;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "coop";
  int* d = nullptr;
  if (hipMalloc(&d, 256 * sizeof(int)) != hipSuccess) return 3;
  hipError_t e;
  if (strcmp(mode, "plain") == 0) {
    hipLaunchKernelGGL(k_touch, dim3(256), dim3(256), 0, 0, d);
    e = hipGetLastError();
  } else {
    void* args[] = {&d};
    e = hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&k_touch), dim3(256), dim3(256), args, 0, 0);
  }
  if (e != hipSuccess) { printf("launch failed: %s\n", hipGetErrorString(e)); return 4; }
  if (hipDeviceSynchronize() != hipSuccess) return 5;
  int h[256];
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 6;
  (void)hipFree(d);
  printf("%s ok: h[255]=%d\n", mode, h[255]);
  return 0;
}
