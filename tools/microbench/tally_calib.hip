// FETCH_SIZE / WRITE_SIZE calibration for the tally kernels' access shapes (MI355X_MICROARCH.md:
// the x2 FETCH_SIZE correction is calibrated for 16-B-per-lane streaming reads only; "other access
// widths are uncalibrated: calibrate on a known byte count in your own access pattern").  The
// tally (kernels_flow.hip) reads 1- and 4-byte vote columns, the 16-word signature columns, and
// touches one 16-byte TallyCell per vote at a random (set, validator) slot of a 16 MB cell array
// (C2's 1M cells; the vote order is shuffled) with loads, a 64-bit atomicMin and a 4-byte store.
// Each shape runs once over 1M votes after a 1 GiB streaming flush (the cells are cold in the
// tally too: K1b gathers GBs of tables between two batches' tallies).  The program prints the
// exact useful bytes and the distinct 128-B lines of each shape; rocprofv3 --pmc FETCH_SIZE and
// --pmc WRITE_SIZE (separate runs) give the counters per dispatch (tools/profile/r3_calib.sh).
// Build: hipcc --offload-arch=gfx950 -O3 tally_calib.hip -o tally_calib
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <set>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Cell { unsigned long long cand; uint32_t acc, row; };

__global__ void flush(const uint4* __restrict__ p, size_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) { const uint4 v = p[i]; acc ^= v.x ^ v.w; }
  if (acc == 0x9e3779b9u) out[0] = acc;
}
__global__ void col_u32_rd(const uint32_t* __restrict__ a, uint32_t n, uint32_t* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n && a[i] == 0x9e3779b9u) out[0] = i;
}
__global__ void col_u8_rd(const uint8_t* __restrict__ a, uint32_t n, uint32_t* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n && a[i] == 0xA5) out[0] = i;
}
__global__ void sig16_rd(const uint32_t* __restrict__ s, uint32_t n, uint32_t* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t d = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) d ^= s[(size_t)j * n + i];
  if (d == 0x9e3779b9u) out[0] = i;
}
__global__ void col_u32_wr(uint32_t* a, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) a[i] = i;
}
__global__ void col_u8_wr(uint8_t* a, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) a[i] = (uint8_t)i;
}
// tally_min's cell access: acc load, then atomicMin on cand
__global__ void cell_min(Cell* c, const uint32_t* __restrict__ idx, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  Cell& x = c[idx[i]];
  if (x.acc == 0) atomicMin(&x.cand, (unsigned long long)i);
}
// tally_resolve's: acc + cand loads, row store
__global__ void cell_resolve(Cell* c, const uint32_t* __restrict__ idx, uint32_t n) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  Cell& x = c[idx[i]];
  if (x.acc == 0 && (uint32_t)x.cand == i) x.row = i + 1;
}
// the cell load alone
__global__ void cell_rd(const Cell* __restrict__ c, const uint32_t* __restrict__ idx, uint32_t n, uint32_t* out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const Cell x = c[idx[i]];
  if (x.acc == 0x9e3779b9u) out[0] = i;
}

int main() {
  const uint32_t n = 1u << 20, n_cells = 1000000;      // C2: 10000 sets x 100 validators
  const size_t flush_bytes = 1ull << 30;
  std::vector<uint32_t> idx(n);
  std::mt19937 rng(7);
  std::vector<uint32_t> perm(n_cells);
  std::iota(perm.begin(), perm.end(), 0u);
  std::shuffle(perm.begin(), perm.end(), rng);
  for (uint32_t i = 0; i < n; ++i) idx[i] = perm[i % n_cells];   // every cell once, then 48576 again
  std::set<uint64_t> lines;
  for (uint32_t i = 0; i < n; ++i) lines.insert((uint64_t)idx[i] * 16 / 128);
  uint4* fl; uint32_t *a32, *sig, *didx, *out; uint8_t* a8; Cell* cells;
  CHK(hipMalloc(&fl, flush_bytes)); CHK(hipMemset(fl, 1, flush_bytes));
  CHK(hipMalloc(&a32, (size_t)n * 4)); CHK(hipMemset(a32, 0, (size_t)n * 4));
  CHK(hipMalloc(&a8, n)); CHK(hipMemset(a8, 0, n));
  CHK(hipMalloc(&sig, (size_t)n * 64)); CHK(hipMemset(sig, 0, (size_t)n * 64));
  CHK(hipMalloc(&cells, (size_t)n_cells * 16)); CHK(hipMemset(cells, 0xff, (size_t)n_cells * 16));
  CHK(hipMalloc(&didx, (size_t)n * 4)); CHK(hipMemcpy(didx, idx.data(), (size_t)n * 4, hipMemcpyHostToDevice));
  CHK(hipMalloc(&out, 64));
  const dim3 g(n / 256), b(256);
  auto fl_ = [&] { hipLaunchKernelGGL(flush, dim3(4096), b, 0, 0, fl, flush_bytes / 16, out); };
  for (int rep = 0; rep < 3; ++rep) {
    fl_(); hipLaunchKernelGGL(col_u32_rd, g, b, 0, 0, a32, n, out);
    fl_(); hipLaunchKernelGGL(col_u8_rd, g, b, 0, 0, a8, n, out);
    fl_(); hipLaunchKernelGGL(sig16_rd, g, b, 0, 0, sig, n, out);
    fl_(); hipLaunchKernelGGL(col_u32_wr, g, b, 0, 0, a32, n);
    fl_(); hipLaunchKernelGGL(col_u8_wr, g, b, 0, 0, a8, n);
    fl_(); hipLaunchKernelGGL(cell_rd, g, b, 0, 0, cells, didx, n, out);
    CHK(hipMemset(cells, 0, (size_t)n_cells * 16));
    fl_(); hipLaunchKernelGGL(cell_min, g, b, 0, 0, cells, didx, n);
    fl_(); hipLaunchKernelGGL(cell_resolve, g, b, 0, 0, cells, didx, n);
  }
  CHK(hipDeviceSynchronize());
  printf("{\"votes\": %u, \"cells\": %u, \"cell_lines_128B\": %zu,\n", n, n_cells, lines.size());
  printf(" \"useful_bytes\": {\"col_u32_rd\": %u, \"col_u8_rd\": %u, \"sig16_rd\": %u, \"col_u32_wr\": %u, \"col_u8_wr\": %u,\n",
         n * 4, n, n * 64, n * 4, n);
  printf("   \"cell_rd\": %u, \"cell_min_idx\": %u, \"cell_resolve_idx\": %u},\n", n * 16 + n * 4, n * 4, n * 4);
  printf(" \"note\": \"cell_* also read the 4 MB index column; cell lines = distinct 128-B lines of the 16 MB array\"}\n");
  return 0;
}
