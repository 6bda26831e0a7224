// Why fusing several multiply-adds into ONE inline-asm statement gave wrong products inside the
// library kernels (csrc/field.hpp mac32 note).  Compile-only probe:
//   hipcc --offload-arch=gfx950 -O3 -c tools/probes/asm_clobber.hip --save-temps
// and read the two kernels' v_mad_u64_u32 pairs.  In k (no early clobber on the read-write
// accumulators) hipcc gives acc0 the same VGPR as the input `a` -- legal for a "+v" operand,
// because asm operands are assumed to be read before any output is written -- so the SECOND
// instruction reads the first one's result where it expects `a`:
//     v_mad_u64_u32 v[2:3], s[0:1], v2, v4, v[2:3]     ; acc0 (= v[2:3]) overwrites v2 = a
//     v_mad_u64_u32 v[4:5], s[2:3], v2, s2, v[4:5]     ; reads the clobbered v2
// With "+&v" / "=&s" (k_ec) every output gets registers of its own (v[6:7], v[8:9]).  Whether
// an accumulator aliases an input depends on the surrounding register allocation, which is why
// the isolated probe was right and the library kernels were not.  Rule: in a multi-instruction
// asm statement every output written before a later instruction reads an input -- accumulators
// and SGPR carries alike -- must be early-clobber.
#include <hip/hip_runtime.h>
#include <cstdint>
// two chained multiply-accumulates in ONE asm statement, second one reading a uniform (SGPR) operand
#define FUSED(acc0, acc1, a, b, s) asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\tv_mad_u64_u32 %1, %3, %4, %6, %1" \
    : "+v"(acc0), "+v"(acc1), "=s"(c0), "=s"(c1) : "v"(a), "v"(b), "s"(s))
#define FUSED_EC(acc0, acc1, a, b, s) asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\tv_mad_u64_u32 %1, %3, %4, %6, %1" \
    : "+&v"(acc0), "+&v"(acc1), "=&s"(c0), "=&s"(c1) : "v"(a), "v"(b), "s"(s))
__global__ void k(uint64_t* o, const uint32_t* x, uint64_t su) {
  uint64_t c0, c1;
  uint32_t a = x[threadIdx.x], b = x[threadIdx.x + 64];
  uint64_t acc0 = a, acc1 = b;
  uint32_t s = (uint32_t)su;   // uniform value in an SGPR, dead after the asm
  FUSED(acc0, acc1, a, b, s);
  o[threadIdx.x] = acc0 ^ acc1;
}
__global__ void k_ec(uint64_t* o, const uint32_t* x, uint64_t su) {
  uint64_t c0, c1;
  uint32_t a = x[threadIdx.x], b = x[threadIdx.x + 64];
  uint64_t acc0 = a, acc1 = b;
  uint32_t s = (uint32_t)su;
  FUSED_EC(acc0, acc1, a, b, s);
  o[threadIdx.x] = acc0 ^ acc1;
}
