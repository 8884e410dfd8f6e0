// One VMM handle mapped at several VAs through HIP (the arena's alias view plus
// stable VAs of managed ranges): does hipMemUnmap of one VA leave the others
// mapped, and do HIP copies on each VA still address the right bytes? Host-side
// checks first (ROCr's own mapping table via hsa_amd_vmem_retain_alloc_handle,
// HIP's via hipMemGetAddressRange); a VA is read by the GPU only when ROCr
// still reports it mapped.
//   hipcc --offload-arch=gfx950 -O2 tools/probe_vmm_multimap.hip -lhsa-runtime64 -o /tmp/probe_vmm_multimap
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

constexpr size_t kSz = 2u << 20;

static void* reserve() {
  void* va = nullptr;
  CK(hipMemAddressReserve(&va, kSz, kSz, nullptr, 0));
  return va;
}
static void map(void* va, hipMemGenericAllocationHandle_t h) {
  CK(hipMemMap(va, kSz, 0, h, 0));
  hipMemAccessDesc ad = {};
  ad.location.type = hipMemLocationTypeDevice;
  ad.location.id = 0;
  ad.flags = hipMemAccessFlagsProtReadWrite;
  CK(hipMemSetAccess(va, kSz, &ad, 1));
}
// ROCr's view: is `va` mapped (it can hand out the handle behind it)?
static bool rocr_mapped(void* va) {
  hsa_amd_vmem_alloc_handle_t h;
  if (hsa_amd_vmem_retain_alloc_handle(&h, va) != HSA_STATUS_SUCCESS) return false;
  hsa_amd_vmem_handle_release(h);
  return true;
}
static void hip_range(const char* what, void* va) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)va);
  std::printf("  %-8s %p: rocr_mapped=%d hip_range=%s base=%p size=%zu%s\n", what, va, (int)rocr_mapped(va),
              e == hipSuccess ? "ok" : hipGetErrorString(e), (void*)base, size,
              (e == hipSuccess && base != va) ? "  <-- HIP attributes this VA to another mapping" : "");
  if (e != hipSuccess) (void)hipGetLastError();
}
// Read 4 bytes at offset 4096 through a HIP copy (only when ROCr maps the VA).
static int hip_read(void* va) {
  if (!rocr_mapped(va)) return -12345;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)va) != hipSuccess || base != va) {
    (void)hipGetLastError();
    return -777;  // HIP would address another mapping: not read (could fault)
  }
  int v = 0;
  hipError_t e = hipMemcpy(&v, (char*)va + 4096, 4, hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return -999;
  }
  return v;
}

int main() {
  CK(hipSetDevice(0));
  if (hsa_init() != HSA_STATUS_SUCCESS) return 1;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemGenericAllocationHandle_t h;
  CK(hipMemCreate(&h, kSz, &prop, 0));
  void *A = reserve(), *X = reserve(), *Y = reserve();
  map(A, h);
  int pat = 0x5a5a1234;
  CK(hipMemset(A, 0, kSz));
  CK(hipMemcpy((char*)A + 4096, &pat, 4, hipMemcpyHostToDevice));
  std::printf("1) alias A mapped\n");
  hip_range("A", A);
  map(X, h);
  std::printf("2) + stable X -> same handle\n");
  hip_range("A", A);
  hip_range("X", X);
  std::printf("   reads: A=%#x X=%#x (want %#x)\n", hip_read(A), hip_read(X), pat);
  map(Y, h);
  std::printf("3) + stable Y -> same handle\n");
  hip_range("A", A);
  hip_range("X", X);
  hip_range("Y", Y);
  std::printf("   reads: A=%#x X=%#x Y=%#x\n", hip_read(A), hip_read(X), hip_read(Y));
  CK(hipMemUnmap(X, kSz));
  std::printf("4) hipMemUnmap(X)\n");
  hip_range("A", A);
  hip_range("X", X);
  hip_range("Y", Y);
  std::printf("   reads: A=%#x Y=%#x\n", hip_read(A), hip_read(Y));
  CK(hipMemUnmap(Y, kSz));
  std::printf("5) hipMemUnmap(Y)\n");
  hip_range("A", A);
  hip_range("Y", Y);
  std::printf("   reads: A=%#x\n", hip_read(A));
  // Two mappings only (alias + one stable VA, remapped one at a time): the
  // round-2 discipline.
  map(X, h);
  CK(hipMemUnmap(X, kSz));
  map(Y, h);
  std::printf("6) map X, unmap X, map Y\n");
  hip_range("A", A);
  hip_range("Y", Y);
  std::printf("   reads: A=%#x Y=%#x\n", hip_read(A), hip_read(Y));
  if (rocr_mapped(Y)) CK(hipMemUnmap(Y, kSz));
  if (rocr_mapped(A)) (void)hipMemUnmap(A, kSz);
  std::printf("done\n");
  return 0;
}
