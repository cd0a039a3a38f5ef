// ed25519_dev.h — per-lane ed25519 building blocks shared by the verify, table-build,
// keygen and sign kernels.
//
// Verification follows golang.org/x/crypto/ed25519.Verify @c2843e01d9a2 (external; the
// reference calls it at types/tx_vote.go:115 via tendermint PubKeyEd25519.VerifyBytes):
//   reject len(sig) != 64 | sig[63] & 0xE0 | undecodable A | s >= L,
//   k = SHA-512(R || A || M) mod L, accept iff encode([s]B + [k](-A)) == R bytewise.
// The double scalar multiplication is evaluated doubling-free over fixed-base radix-16
// tables (ge.h Niels entries): T_P[i][j] = j * 16^i * P for i < 64, j <= 8 (j = 0 the
// identity), so [s]B + [k](-A) = sum_i T_B[i][s_i] - T_A[i][k_i] with signed digits.
// This is exact group arithmetic, hence the same point and encoding as x/crypto's
// sliding-window GeDoubleScalarMultVartime.
#pragma once
#include "fe.h"
#include "sc.h"
#include "sha2.h"
#include "ge.h"

namespace txv {

constexpr int kTabPositions = 64;      // radix-16 digits of a 253-bit scalar
constexpr int kTabEntries = 9;         // |digit| in 0..8 (0 = identity)
constexpr int kEntryWords = 24;        // y+x, y-x, 2dxy: 3 x 8 limbs
constexpr int kTableWords = kTabPositions * kTabEntries * kEntryWords;   // 13824 words = 55296 B

// message words are stored big-endian (SHA-native), zero beyond the message length.
// Hash-input word gw of (prefix || M || padding) with a prefix of `pre_words` 64-bit words.
struct MsgView {
  const uint64_t* words;   // column base for this lane: words[w * stride]
  uint32_t stride;         // column stride (in u64 words)
  uint32_t n_words;        // stored words per message
  uint32_t len;            // message length in bytes
};

TXV_HD uint64_t msg_word(const MsgView& m, uint32_t w) {
  return w < m.n_words ? m.words[(size_t)w * m.stride] : 0ull;
}

// number of 128-byte SHA-512 blocks for prefix_bytes + len
TXV_HD uint32_t sha512_nblocks(uint32_t total_len) { return (total_len + 17u + 127u) / 128u; }

// SHA-512 of pre[0..pre_words) || M, pre given as big-endian words.  Result as 16
// little-endian u32 limbs of the 512-bit digest interpreted little-endian (ScReduce input).
TXV_HD void sha512_prefixed(uint32_t digest_le[16], const uint64_t* pre, int pre_words, const MsgView& m) {
  uint64_t st[8];
  sha512_init(st);
  const uint32_t total = 8u * (uint32_t)pre_words + m.len;
  const uint32_t nblk = sha512_nblocks(total);
  const uint32_t pad_word = total >> 3, pad_shift = 56u - 8u * (total & 7u);
  const uint32_t last = 16u * nblk - 1u;
  for (uint32_t b = 0; b < nblk; ++b) {
    uint64_t w[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      uint32_t gw = 16u * b + (uint32_t)t;
      uint64_t v;
      if (b == 0 && t < pre_words) v = pre[t];
      else v = msg_word(m, gw - (uint32_t)pre_words);
      if (gw == pad_word) v |= 0x80ull << pad_shift;
      if (gw == last) v = (uint64_t)total * 8u;
      w[t] = v;
    }
    sha512_block(st, w);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    digest_le[2 * k] = bswap32((uint32_t)(st[k] >> 32));
    digest_le[2 * k + 1] = bswap32((uint32_t)st[k]);
  }
}

// table entry fetch: T[pos][idx] from a flat word array
template <typename Ptr>
TXV_HD ge_niels load_entry(Ptr tab, int pos, int idx) {
  const int base = (pos * kTabEntries + idx) * kEntryWords;
  ge_niels e;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    e.ypx.v[i] = tab[base + i];
    e.ymx.v[i] = tab[base + 8 + i];
    e.xy2d.v[i] = tab[base + 16 + i];
  }
  return e;
}

// sum_i T_B[i][s_i] + T_A[i][-k_i]   (negA: digits of k are negated, giving [k](-A))
template <typename PtrB, typename PtrA>
TXV_HD ge_ext double_scalarmult_fixed(PtrB tb, PtrA ta, const uint32_t s_packed[8],
                                      const uint32_t k_packed[8], bool use_a) {
  ge_ext P = ge_identity();
  uint32_t ps[8], pk[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { ps[i] = s_packed[i]; pk[i] = k_packed[i]; }
  for (int w = 0; w < 8; ++w) {
    const uint32_t ws = ps[0], wk = pk[0];
#pragma unroll
    for (int i = 0; i < 7; ++i) { ps[i] = ps[i + 1]; pk[i] = pk[i + 1]; }
    for (int j = 0; j < 8; ++j) {
      const int pos = 8 * w + j;
      const int ds = sc_nibble(ws, j);
      P = ge_madd(P, load_entry(tb, pos, ds < 0 ? -ds : ds), ds < 0);
      if (use_a) {
        const int dk = sc_nibble(wk, j);
        P = ge_madd(P, load_entry(ta, pos, dk < 0 ? -dk : dk), dk > 0);
      }
    }
  }
  return P;
}

// the base point's canonical encoding (little-endian words)
TXV_HD void base_point_words(uint32_t w[8]) {
  const uint32_t b[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                         0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = b[i];
}

}  // namespace txv
