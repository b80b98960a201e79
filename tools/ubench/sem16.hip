// Semantics probe: what do 16-bit VOP2 ops and v_pack_b32_f16 do to a full
// 32-bit register (upper half zeroed / preserved; NaN/denormal bit patterns)?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
__global__ void k(const uint32_t *in, uint32_t *out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x = in[i], y = in[(i + 1) % n];
  uint32_t a = y, b = y, c, d = y, e = y;
  asm volatile("v_lshlrev_b16 %0, 3, %1" : "+v"(a) : "v"(x));
  asm volatile("v_pack_b32_f16 %0, %1, %1 op_sel:[1,0,0]" : "=v"(c) : "v"(x));
  uint32_t m80 = 0x80; asm volatile("v_mad_u16 %0, %1, %3, %2 op_sel:[0,0,0,1]" : "+v"(d) : "v"(x), "v"(y), "v"(m80));
  asm volatile("v_lshrrev_b16 %0, 3, %1" : "+v"(b) : "v"(x));
  asm volatile("v_bitop3_b16 %0, %1, %2, %1 bitop3:0xf0 op_sel:[0,0,0,1]" : "+v"(e) : "v"(x), "v"(y));
  out[5 * i + 0] = a; out[5 * i + 1] = b; out[5 * i + 2] = c; out[5 * i + 3] = d; out[5 * i + 4] = e;
}
int main() {
  const int n = 1 << 20;
  uint32_t *h = (uint32_t *)malloc(4 * n), *o = (uint32_t *)malloc(20 * n);
  uint64_t s = 12345;
  for (int i = 0; i < n; ++i) { s = s * 6364136223846793005ull + 1442695040888963407ull; h[i] = (uint32_t)(s >> 32); }
  h[0] = 0x7c017c01; h[1] = 0x00010001; h[2] = 0xfe00fe00; h[3] = 0x7fff8001;
  uint32_t *din, *dout; (void)hipMalloc(&din, 4 * n); (void)hipMalloc(&dout, 20 * n);
  (void)hipMemcpy(din, h, 4 * n, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(din, dout, n);
  (void)hipMemcpy(o, dout, 20 * n, hipMemcpyDeviceToHost);
  int bad[5] = {0};
  int hi_zero_a = 0, hi_pres_a = 0;
  for (int i = 0; i < n; ++i) {
    uint32_t x = h[i], y = h[(i + 1) % n];
    uint32_t lo_a = (uint16_t)(x << 3);
    if (o[5 * i] == lo_a) hi_zero_a++;
    if (o[5 * i] == ((y & 0xffff0000u) | lo_a)) hi_pres_a++;
    if ((o[5 * i + 2]) != ((x >> 16) | (x << 16))) bad[2]++;
    uint32_t dexp = (y & 0xffffu) | ((uint32_t)(uint16_t)((x & 0xffff) * 0x80 + (y & 0xffff)) << 16);
    if (o[5 * i + 3] != dexp) bad[3]++;
    if (i < 3) printf("x=%08x y=%08x lshl16=%08x lshr16=%08x pack=%08x mad_hi=%08x (want %08x) bitop3_hi=%08x\n", x, y, o[5*i], o[5*i+1], o[5*i+2], o[5*i+3], dexp, o[5*i+4]);
  }
  printf("lshlrev_b16: upper zeroed %d, upper preserved %d of %d\n", hi_zero_a, hi_pres_a, n);
  printf("pack_b32_f16 swap mismatches %d; mad_u16 dst-hi mismatches %d\n", bad[2], bad[3]);
  return 0;
}
