// Probe of the v_mfma_i32_16x16x64_i8 operand layout on gfx950 (exact integer data): random A, B
// fragments, D compared with candidate lane/byte -> (row, k) maps.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int i32x4 __attribute__((ext_vector_type(4)));
__global__ void k_mfma(const signed char* A, const signed char* B, int* D) {
  const int l = threadIdx.x;
  i32x4 a, b;
  for (int r = 0; r < 4; ++r) {
    a[r] = *(const int*)(A + l * 16 + r * 4);
    b[r] = *(const int*)(B + l * 16 + r * 4);
  }
  i32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = c[r];
}
static int kmap(int hyp, int l, int b) {
  if (hyp == 0) return 16 * (l >> 4) + b;                         // contiguous 16 per lane group
  if (hyp == 1) return 8 * (l >> 4) + (b & 7) + 32 * (b >> 3);     // two 8-byte halves 32 apart
  return 4 * (l >> 4) + (b & 3) + 16 * (b >> 2);                   // four 4-byte quarters
}
int main() {
  signed char *A, *B;
  int* D;
  if (hipMallocManaged(&A, 1024) || hipMallocManaged(&B, 1024) || hipMallocManaged(&D, 1024)) return 1;
  srand(1);
  for (int i = 0; i < 1024; ++i) { A[i] = (signed char)(rand() % 15 - 7); B[i] = (signed char)(rand() % 15 - 7); }
  hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, A, B, D);
  if (hipDeviceSynchronize()) return 2;
  for (int hyp = 0; hyp < 3; ++hyp) {
    int a[16][64], bm[64][16], bad = 0;
    for (int l = 0; l < 64; ++l)
      for (int b = 0; b < 16; ++b) {
        a[l & 15][kmap(hyp, l, b)] = A[l * 16 + b];
        bm[kmap(hyp, l, b)][l & 15] = B[l * 16 + b];
      }
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * (l >> 4) + r, col = l & 15;
        int s = 0;
        for (int k = 0; k < 64; ++k) s += a[row][k] * bm[k][col];
        bad += s != D[l * 4 + r];
      }
    printf("hypothesis %d: %d / 256 mismatches\n", hyp, bad);
  }
  // the symmetric-split property the conv kernel relies on: product of lo halves + hi halves
  return 0;
}
