// Localisation by tile dedup + bucket partition ("tp", mixed key spaces <= 34 bits).
//
// Reference: Localizer::countUniqIndex / remapIndex (src/util/localizer.h:69-191) sort
// every (key, position) pair of a minibatch and rebuild a CSR with local ids.
//
// Measured on MI355X for a 65,536 x 39 Criteo-shaped minibatch (2.56 M keys, 234 K
// distinct): 1 944 hot keys hold 77 % of the occurrences, and a full LSD radix sort
// (sort32.hip) is 16 small launches, ~200 us. Device-scope atomics run at ~20 per
// ns (benchmarks/probe_atomics.py), so a global hash with per-key atomics cannot beat
// it either. This path touches each occurrence once, in LDS, and works on the
// tile-distinct "entries" (~1 M) afterwards, with no global atomics at all:
//
//   tile     one 512-thread workgroup per tile of 8192 occurrences: mix, LDS hash
//            dedup, counting sort of the tile's distinct keys by bucket (top BB key
//            bits) -> tkeys[tile][pos], per-tile bucket offsets toff[tile][b],
//            rep[i] = tile entry of occurrence i (u16)
//   bucket   one workgroup per bucket: gather the bucket's entries from every tile
//            (a key occurs at most once per tile, so a hot key is <= #tiles entries
//            and buckets stay balanced), LDS hash -> distinct keys + entry counts,
//            rank sort of the distinct keys; the bucket's global unique / entry bases
//            by a decoupled look-back over the earlier buckets' published counts;
//            then uniq, seg_start (over entries), the entry CSC (pos_s = entry id,
//            segid) and ent_uid[entry] = unique id, straight from LDS
//   gather   local_col[i] = ent_uid[tile * 8192 + rep[i]]
// Backward: per tile, LDS float accumulation of coef[row] * val into its entries
// (psum), then a 64-lane segmented scan of psum over the entry CSC.
//
// Buckets are ranges of the mixed key space, so the unique keys come out sorted
// (the multi-GPU owner split and the ordered home slots of the KV table rely on it).
#include "countmin.cuh"
#include "kv_slot.cuh"
#include "loss.cuh"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace psamd {

namespace tp {
constexpr int kThr = 1024;              // tile workgroup
// 8192 occurrences per tile (a 65,536 x 39 minibatch is 313 tiles). Measured and not
// kept: 10,240 (250 tiles, at most one per CU): tile 24.7 -> 24.2 us and fused
// forward+backward 24.3 -> 23.7, but 136 / 87 KB of LDS per workgroup left no room for
// the other streams' kernels and the pipelined step went 0.118 -> 0.126 ms
// (profiles/r3_tile_count.log).
constexpr int kIt = 8;
constexpr int kTile = kThr * kIt;       // 8192 occurrences
constexpr int kHash = 2 * kTile;        // LDS hash slots of a tile (load <= 0.5)
constexpr int kHB = 14;                 // log2 kHash
// Quotient encoding of the tile hash: a key k (<= 34 bits, uniformly mixed) probes from
// home slot k mod kHash, and the slot keeps (k >> kHB) << kDispB | displacement, which
// with the slot index gives k back: 34-bit keys in 32-bit LDS words.
constexpr int kDispB = 12;
constexpr uint32_t kMaxDisp = (1u << kDispB) - 1;  // never reached at load <= 0.5
constexpr int kMaxBk = 2048;            // buckets (tile LDS: 72 KB -> 2 workgroups per CU)
constexpr int kMaxT = 640;              // tiles (n <= 5.2 M)
constexpr int kBThr = 256;              // emit workgroups
constexpr int kBkThr = 512;             // bucket workgroups
constexpr int kECap = 4096;             // entries of one bucket (global stride)
constexpr int kECapL = 4064;            // ... held in LDS (bucket kernel LDS <= 40 KB:
                                        // 4 workgroups per CU instead of 3)
constexpr int kDH = 2048;               // distinct-key hash of one bucket
constexpr int kBkProbe = 128;           // probe chain bound of the bucket hash build
constexpr uint32_t kEmpty = 0xffffffffu;
}  // namespace tp

__device__ __forceinline__ uint32_t tp_hash(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

template <int kN>
__device__ __forceinline__ uint32_t tp_block_scan(uint32_t v, uint32_t* lds, uint32_t* total) {
  constexpr int kW = kN / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0;
    for (int w = 0; w < kW; ++w) {
      const uint32_t t = lds[w];
      lds[w] = run;
      run += t;
    }
    lds[kW] = run;
  }
  __syncthreads();
  const uint32_t r = x - v + lds[wid];
  *total = lds[kW];
  __syncthreads();
  return r;
}

// sum of a[0:b) by one workgroup (a few thousand L2-resident words)
template <int kN>
__device__ __forceinline__ uint32_t tp_prefix(const uint32_t* __restrict__ a, int b, uint32_t* lds) {
  uint32_t s = 0;
  for (int i = threadIdx.x; i < b; i += kN) s += a[i];
  uint32_t tot;
  tp_block_scan<kN>(s, lds, &tot);
  return tot;
}

__device__ __forceinline__ uint64_t tp_match_any(uint32_t v, int nbits, uint64_t active) {
  uint64_t peers = active;
  for (int b = 0; b < nbits; ++b) {
    const bool bit = (v >> b) & 1u;
    const uint64_t bal = __ballot(bit);
    peers &= bit ? bal : ~bal;
  }
  return peers;
}

// ------------------------------------------------------------------------ tile
// Phase marks of the tile kernel (a tuning aid, benchmarks/prof_tile_phases.py): null
// unless tp_tile_set_prof() installed a buffer of 16 u64 per workgroup.
__device__ uint64_t* g_tile_prof = nullptr;
#define TILE_MARK(k)                                                            \
  if (tpp && threadIdx.x == 0) tpp[(int64_t)blockIdx.x * 16 + (k)] = clock64()

// kQuot = false (<= 31-bit keys): the slot keeps the key itself, home = low kHB key bits;
// kQuot = true (32..34 bits): quotient encoding, home = low kHB key bits.
// kCnt (the tail filter's counts): ecnt[tile * kTile + e] = occurrences of entry e in the
// tile, saturated to a byte (LDS u16 pairs in the dead hash, one integer LDS add per
// occurrence).
// (8 waves per SIMD = 2 workgroups per CU: <= 64 VGPRs. The quotient variant compiled to
// 66 without the bound, i.e. 1 workgroup per CU: localise 90 vs 80 us.)
template <bool kQuot, bool kCnt = false>
__global__ void __launch_bounds__(tp::kThr, 8)
tp_tile_kernel(const uint64_t* __restrict__ raw, int64_t n, KeyMix m, int shift, int nbk,
               uint32_t* __restrict__ tkeys, uint16_t* __restrict__ toff,
               int32_t* __restrict__ dcnt, uint16_t* __restrict__ rep,
               int32_t* __restrict__ err, int lts, uint8_t* __restrict__ ecnt = nullptr) {
  using namespace tp;
  __shared__ uint32_t hk[kHash];    // quotient-encoded keys; after the bucket sort: entry position
  __shared__ uint32_t cnt[kMaxBk];  // per-bucket counts, then offsets
  __shared__ uint32_t lds[kThr / 64 + 1];
  const int t = threadIdx.x;
  uint64_t* const tpp = g_tile_prof;
  if (tpp && t == 0) tpp[(int64_t)blockIdx.x * 16 + 8] = __builtin_amdgcn_s_memrealtime();
  TILE_MARK(0);
  for (int i = t; i < kHash; i += kThr) hk[i] = kEmpty;
  for (int d = t; d < nbk; d += kThr) cnt[d] = 0;
  __syncthreads();
  TILE_MARK(1);
  // occurrences [base, base + lim) (2^lts per tile, tp_geom); entry ids keep the
  // kTile stride (tkeys, dcnt, the consumers' tile * kTile + entry)
  const int64_t base = (int64_t)blockIdx.x << lts;
  const int lim = (int)(n - base < (1 << lts) ? n - base : (1 << lts));
  uint64_t kr[kIt];  // raw keys, then the mixed keys
  uint16_t sl[kIt];  // hash slot of every key
  uint32_t rr[kIt];  // a key this lane inserted (one lane per distinct key): rank in its
                     // bucket, then its entry position; kEmpty otherwise
  uint32_t won = 0;  // bit j: this lane inserted key j
  bool bad = false;
#pragma unroll
  for (int j = 0; j < kIt; ++j) {  // all loads in flight before the LDS insert chain
    const int o = j * kThr + t;
    kr[j] = o < lim ? raw[base + o] : 0ull;
  }
  if (tpp) {  // (profiling only: every load landed, workgroup-wide)
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    TILE_MARK(2);
  }
  // (<= 31 bits: the mix in 32-bit arithmetic -- the low bits of a product depend only
  // on the low bits of its factors, so it equals mix_key -- and the mixed key's own low
  // bits as the home slot: ~12 fewer VALU per key than the 64-bit mix + tp_hash. Measured
  // and not kept: two keys per probe loop, both probes' LDS reads and CAS in flight
  // together: insert phase 19.1 -> 22.2 k cycles per workgroup, benchmarks/prof_tile_phases.py)
#pragma unroll
  for (int j = 0; j < kIt; ++j) {
    sl[j] = 0;
    if (j * kThr + t < lim) {
      const uint64_t k = kQuot ? mix_key(kr[j], m) : (uint64_t)mix_key32(kr[j], m);
      kr[j] = k;
      const uint32_t q = kQuot ? (uint32_t)(k >> kHB) << kDispB : (uint32_t)k;
      uint32_t h = (uint32_t)k & (kHash - 1);
      uint32_t d = 0;
      for (; d < kMaxDisp; ++d) {  // slot h holds key k iff it holds q | d (q: kQuot = false)
        const uint32_t want = kQuot ? q | d : q;
        const uint32_t cur = hk[h];
        if (cur == want) break;
        if (cur == kEmpty) {
          const uint32_t prev = atomicCAS(&hk[h], kEmpty, want);
          if (prev == kEmpty) {
            won |= 1u << j;
            break;
          }
          if (prev == want) break;
        }
        h = (h + 1) & (kHash - 1);
      }
      bad |= d == kMaxDisp;
      sl[j] = (uint16_t)h;
    }
  }
  // counting sort of the distinct keys by bucket (top key bits), by the lanes that
  // inserted them: their keys are in registers, so no pass over the (mostly empty) hash
  // (the earlier form scanned all 16 K slots twice: ~3 K of them hold a key). The tile
  // keys leave as their low `shift` bits (the bucket holds the rest).
#pragma unroll
  for (int j = 0; j < kIt; ++j)
    rr[j] = (won >> j) & 1u ? atomicAdd(&cnt[kr[j] >> shift], 1u) : kEmpty;
  if (bad && err) atomicOr(err, 2);
  __syncthreads();
  TILE_MARK(3);
  // exclusive scan of the bucket counts (nbk <= kMaxBk: 2 per thread)
  constexpr int kDP = kMaxBk / kThr;
  uint32_t c[kDP], s = 0;
#pragma unroll
  for (int e = 0; e < kDP; ++e) {
    const int d = t * kDP + e;
    c[e] = d < nbk ? cnt[d] : 0u;
    s += c[e];
  }
  uint32_t D;
  uint32_t run = tp_block_scan<kThr>(s, lds, &D);
  uint16_t* to = toff + (int64_t)blockIdx.x * (nbk + 1);
#pragma unroll
  for (int e = 0; e < kDP; ++e) {
    const int d = t * kDP + e;
    if (d < nbk) {
      cnt[d] = run;
      to[d] = (uint16_t)run;
    }
    run += c[e];
  }
  if (t == 0) {
    to[nbk] = (uint16_t)D;
    dcnt[blockIdx.x] = (int32_t)D;
  }
  __syncthreads();
  TILE_MARK(4);
  // each inserted key -> its entry position: tile key out, and its hash slot now holds
  // the position (no lane reads hk between the two barriers)
  uint32_t* tk = tkeys + (int64_t)blockIdx.x * kTile;
  const uint64_t smask = (1ull << shift) - 1;
#pragma unroll
  for (int j = 0; j < kIt; ++j) {
    if (rr[j] != kEmpty) {
      const uint32_t pos = cnt[kr[j] >> shift] + rr[j];
      tk[pos] = (uint32_t)(kr[j] & smask);
      hk[sl[j]] = pos;
    }
  }
  __syncthreads();
  TILE_MARK(5);
#pragma unroll
  for (int j = 0; j < kIt; ++j) {
    const int o = j * kThr + t;
    if (o < lim) {
      const uint16_t pos = (uint16_t)hk[sl[j]];
      rep[base + o] = pos;
      if (kCnt) sl[j] = pos;
    }
  }
  if (kCnt) {  // occurrences per entry: u16 pairs in the dead hash
    __syncthreads();
    for (uint32_t i = t; i < (D + 1) / 2; i += kThr) hk[i] = 0u;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kIt; ++j)
      if (j * kThr + t < lim) atomicAdd(&hk[sl[j] >> 1], 1u << ((sl[j] & 1) * 16));
    __syncthreads();
    uint8_t* ec = ecnt + (int64_t)blockIdx.x * kTile;
    for (uint32_t i = t; i < D; i += kThr) {
      const uint32_t c = (hk[i >> 1] >> ((i & 1) * 16)) & 0xffffu;
      ec[i] = (uint8_t)(c > 255u ? 255u : c);
    }
  }
  if (tpp && t == 0) {
    TILE_MARK(6);
    tpp[(int64_t)blockIdx.x * 16 + 9] = __builtin_amdgcn_s_memrealtime();
    tpp[(int64_t)blockIdx.x * 16 + 10] = __smid();
  }
}
#undef TILE_MARK

void tp_tile_set_prof(uint64_t* p) {
  PSAMD_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_tile_prof), &p, sizeof(p)));
}

// ---------------------------------------------------------------------- bucket
// One workgroup per COARSE bucket c: the fine buckets 2c and 2c+1 of the tile kernel's
// counting sort (a range of the mixed key space; the two runs of a tile are adjacent,
// so the pair is one run per tile). It dedups the pair AND writes its slice of the
// global outputs:
//   build          the entries from every tile (flat: each thread locates its entries
//                  by binary search over the per-tile run prefix and loads them
//                  together; the entry ids stay in registers), each key (suffix plus the
//                  fine bucket's low bit above it) inserted into an LDS hash with an entry
//                  count, then the occupied slots compacted -> (key | count | slot) list;
//                  the pair's distinct and entry counts are PUBLISHED for the look-back
//   rank sort      distinct keys are unique: rank = number of smaller keys (2 or 4
//                  threads per key when they are few)
//   look-back      one wave derives the bucket's global bases (unique ids, entries) from
//                  the earlier buckets' published counts (decoupled look-back: 64 status
//                  words per step, nearest inclusive prefix ends it) and publishes its
//                  own inclusive prefix
//   starts         prefix of the counts in key order -> uniq, seg_start (global)
//   assign         every entry takes the next position of its key's segment (LDS
//                  atomic: the order inside a segment is not fixed) -> entry CSC
//                  (pos_s, segid), ent_uid
// Pairs: 1024 workgroups of 512 threads at 40 KB of LDS are ONE round on the 256 CUs
// (2048 single buckets were two rounds, 43 us; profiles/r3_tp_phases.log). A pair whose
// entries overflow the LDS capacity (or its hash) falls back to its two fine buckets one
// after the other: count both, publish, look back, then build / sort / write each again.
// The fine geometry (<= 1280 occurrences per fine bucket) keeps that fallback exact even
// when every key is distinct.
// Workgroups are dispatched in blockIdx order, so a bucket only ever waits for buckets
// that are running or done; the spin is bounded anyway (err bit 4, no hang). The status
// words carry an 8-bit launch epoch (device counter, advanced by the last bucket), so
// they need no reset between launches or graph replays.
// Per-phase shader-clock marks (prof != null) are a tuning aid
// (benchmarks/prof_tp_phases.py).
namespace tp {
constexpr uint64_t kStA = 1, kStP = 2;  // status flags: aggregate / inclusive prefix
constexpr uint32_t kStM = (1u << 27) - 1;
constexpr int kG = (kECapL + kBkThr - 1) / kBkThr;  // entries per thread
}  // namespace tp
__device__ __forceinline__ uint64_t tp_status(uint32_t ep, uint64_t flag, uint32_t d, uint32_t e) {
  return ((uint64_t)ep << 56) | (flag << 54) | ((uint64_t)(d & tp::kStM) << 27) | (e & tp::kStM);
}

// Build the dedup state of fine buckets [f0, f0 + nf) (nf = 2: a pair; the key inserted
// is (hb + fine bucket - f0) << shift | suffix). Leaves: eh[g] = hash slot of entry g,
// idx[] = tile entry ids (registers), hkey / hcnt = the hash, dl[0..D) = the compacted
// occupied slots. Returns (block-uniform) whether every entry found a slot within the
// LDS capacity; *E / *D = entries / distinct keys.
template <bool kCnt = false>  // kCnt: hcnt sums the entries' occurrence counts (ecnt)
__device__ __forceinline__ bool tp_bk_build(const uint32_t* __restrict__ tkeys,
                                            const uint16_t* __restrict__ toff, int nbf, int T,
                                            int shift, int f0, int nf, uint32_t hb,
                                            uint32_t* hkey, uint32_t* hcnt, uint64_t* dl,
                                            uint16_t* eh, uint32_t* lds, uint32_t* flag,
                                            int32_t (&idx)[tp::kG], uint32_t* E_out,
                                            uint32_t* D_out, uint64_t* prof,
                                            const uint8_t* __restrict__ ecnt = nullptr) {
  using namespace tp;
  const int t = threadIdx.x;
  uint32_t* tpre = reinterpret_cast<uint32_t*>(dl);                // [kMaxT + 1]
  uint16_t* tlo = reinterpret_cast<uint16_t*>(tpre + kMaxT + 1);  // [kMaxT]
  uint16_t* tmid = tlo + kMaxT;                                   // [kMaxT]
  for (int s = t; s < kDH; s += kBkThr) {
    hkey[s] = kEmpty;
    hcnt[s] = 0;
  }
  if (t == 0) *flag = 0;
  // per-tile runs [toff[q][f0], toff[q][f0 + nf]): thread t owns tiles [t*per, t*per + per)
  const int per = (T + kBkThr - 1) / kBkThr;
  const int q0 = t * per, q1 = q0 + per < T ? q0 + per : T;
  uint32_t c = 0;
  for (int q = q0; q < q1; ++q) {
    const uint16_t* to = toff + (int64_t)q * (nbf + 1);
    const uint32_t lo = to[f0], hi = to[f0 + nf];
    tlo[q] = (uint16_t)lo;
    tmid[q] = (uint16_t)((nf == 2 ? to[f0 + 1] : hi) - lo);
    tpre[q] = hi - lo;
    c += hi - lo;
  }
  uint32_t E;
  uint32_t w = tp_block_scan<kBkThr>(c, lds, &E);
  for (int q = q0; q < q1; ++q) {
    const uint32_t len = tpre[q];
    tpre[q] = w;
    w += len;
  }
  if (t == 0) tpre[T] = E;
  __syncthreads();
  if (prof && t == 0) prof[(int64_t)blockIdx.x * 12 + 1] = clock64();
  const uint32_t En = E < (uint32_t)kECapL ? E : (uint32_t)kECapL;
  bool bad = E > (uint32_t)kECapL;
  uint32_t hib = 0;  // bit q: entry q lies in the pair's second fine bucket
#pragma unroll
  for (int q = 0; q < kG; ++q) {
    const uint32_t g = q * kBkThr + t;
    idx[q] = -1;
    if (g < En) {
      int lo = 0, up = T - 1;  // last tile with tpre[q] <= g
      while (lo < up) {
        const int mid = (lo + up + 1) >> 1;
        if (tpre[mid] <= g) lo = mid; else up = mid - 1;
      }
      const uint32_t off = g - tpre[lo];
      idx[q] = lo * kTile + tlo[lo] + (int32_t)off;
      hib |= (off >= tmid[lo] ? 1u : 0u) << q;
    }
  }
  uint32_t kv[kG];
  uint32_t ecp[(kG + 3) / 4];  // (kCnt: the entries' occurrence counts, 4 bytes a word)
#pragma unroll
  for (int q = 0; q < kG; ++q) kv[q] = idx[q] >= 0 ? tkeys[idx[q]] : 0u;
  if (kCnt) {
#pragma unroll
    for (int w = 0; w < (kG + 3) / 4; ++w) ecp[w] = 0u;
#pragma unroll
    for (int q = 0; q < kG; ++q)
      if (idx[q] >= 0) ecp[q >> 2] |= (uint32_t)ecnt[idx[q]] << ((q & 3) * 8);
  }
#pragma unroll
  for (int q = 0; q < kG; ++q) {
    if (idx[q] < 0) continue;
    const uint32_t g = q * kBkThr + t;
    const uint32_t key = kv[q] | ((hb + ((hib >> q) & 1u)) << shift);
    uint32_t h = tp_hash(key) & (kDH - 1);
    bool ok = false;
    // (another lane gave up: the build is lost anyway)
    bad |= __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0u;
    // (bounded chain: a hash this full -- near-distinct keys -- is cheaper to give up on
    // than to probe through: the overflow form takes the pair, profiles/r6_skew_layout.log)
    for (int p = 0; p < kBkProbe && !bad; ++p) {
      const uint32_t cu = hkey[h];
      if (cu == kEmpty) {
        const uint32_t prev = atomicCAS(&hkey[h], kEmpty, key);
        if (prev == kEmpty || prev == key) { ok = true; break; }
      } else if (cu == key) {
        ok = true;
        break;
      }
      h = (h + 1) & (kDH - 1);
    }
    if (ok) {
      atomicAdd(&hcnt[h], kCnt ? (ecp[q >> 2] >> ((q & 3) * 8)) & 0xffu : 1u);
    } else if (!bad) {
      bad = true;
      atomicOr(flag, 1u);
    }
    eh[g] = ok ? (uint16_t)h : (uint16_t)0xffffu;
  }
  if (bad) atomicOr(flag, 1u);
  __syncthreads();
  if (prof && t == 0) prof[(int64_t)blockIdx.x * 12 + 2] = clock64();
  // compact the occupied slots (strided: conflict-free LDS reads)
  constexpr int kPer = kDH / kBkThr;  // 4
  uint64_t ent[kPer];
  uint32_t cc = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int s = q * kBkThr + t;
    ent[q] = hkey[s] != kEmpty
                 ? (((uint64_t)hkey[s] << 32) |
                    ((uint64_t)(kCnt ? min(hcnt[s], 0xffffu) : hcnt[s]) << 16) | (uint64_t)s)
                 : ~0ull;
    cc += ent[q] != ~0ull;
  }
  uint32_t D;
  uint32_t wd = tp_block_scan<kBkThr>(cc, lds, &D);  // (its barriers: every locate is done)
#pragma unroll
  for (int q = 0; q < kPer; ++q)
    if (ent[q] != ~0ull) dl[wd++] = ent[q];
  *E_out = En;
  *D_out = D;
  const bool good = *flag == 0u;
  __syncthreads();
  return good;
}

// rank sort of dl[0..D) into hs (distinct keys: rank = # smaller keys). Broadcast LDS
// reads, two keys per 16-B read and four reads in flight; dl[D .. D+7] padded with ~0
// (larger than any entry: key < 2^32 in the high word) so the tail needs no test. With
// <= 256 keys, 2 or 4 threads split each key's scan and add their counts in LDS.
__device__ __forceinline__ void tp_bk_ranksort(uint64_t* dl, uint64_t* hs, uint32_t D) {
  using namespace tp;
  const int t = threadIdx.x;
  if (t < 8 && D + t < (uint32_t)kDH) dl[D + t] = ~0ull;
  uint32_t* rk = reinterpret_cast<uint32_t*>(hs + 1024);  // beyond any output rank < 256
  const int tpk = D <= 128 ? 4 : D <= 256 ? 2 : 1;
  if (tpk > 1 && t < 256) rk[t] = 0;
  __syncthreads();
  const uint4* d4 = reinterpret_cast<const uint4*>(dl);
  const uint32_t nq = (D + 7) / 8;
  if (tpk > 1) {
    const int nk = kBkThr / tpk, i = t % nk, h = t / nk;
    const uint32_t pq = (nq + tpk - 1) / tpk;
    const uint32_t qa = h * pq, qb = qa + pq < nq ? qa + pq : nq;
    if ((uint32_t)i < D) {
      const uint64_t x = dl[i];
      uint32_t r = 0;
      for (uint32_t q = qa; q < qb; ++q) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = d4[q * 4 + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          r += (((uint64_t)v[k].y << 32) | v[k].x) < x;
          r += (((uint64_t)v[k].w << 32) | v[k].z) < x;
        }
      }
      atomicAdd(&rk[i], r);
    }
    __syncthreads();
    if (h == 0 && (uint32_t)i < D) hs[rk[i]] = dl[i];
  } else {
    for (uint32_t i = t; i < D; i += kBkThr) {
      const uint64_t x = dl[i];
      uint32_t r = 0;
      for (uint32_t q = 0; q < nq; ++q) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = d4[q * 4 + k];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          r += (((uint64_t)v[k].y << 32) | v[k].x) < x;
          r += (((uint64_t)v[k].w << 32) | v[k].z) < x;
        }
      }
      hs[r] = x;
    }
  }
}

// starts + assign: the sorted keys hs[0..D) -> uniq / seg_start from (ubase, ebase);
// every entry of idx[] takes the next position of its key's segment.
__device__ __forceinline__ void tp_bk_emit(const uint64_t* hs, uint64_t* dl, const uint16_t* eh,
                                           const int32_t (&idx)[tp::kG], uint32_t D,
                                           uint32_t ubase, uint32_t ebase, uint64_t key0,
                                           uint32_t* lds, int32_t* __restrict__ pos_s,
                                           int32_t* __restrict__ segid,
                                           uint64_t* __restrict__ uniq,
                                           int32_t* __restrict__ seg_start,
                                           int32_t* __restrict__ ent_uid,
                                           float* __restrict__ zero_a,
                                           unsigned long long* __restrict__ zero_b,
                                           int64_t u_cap, int64_t e_cap, uint64_t* prof) {
  using namespace tp;
  const int t = threadIdx.x;
  uint32_t* cur = reinterpret_cast<uint32_t*>(dl);        // [kDH] per slot
  uint16_t* jj = reinterpret_cast<uint16_t*>(cur + kDH);  // [kDH] per slot
  __syncthreads();  // (dl: the rank sort's source is dead)
  uint32_t carry = 0;
  for (uint32_t j0 = 0; j0 < D; j0 += kBkThr) {
    const uint32_t j = j0 + t;
    const uint64_t v = j < D ? hs[j] : 0ull;
    const uint32_t cnt = (uint32_t)(v >> 16) & 0xffffu;
    uint32_t tot;
    const uint32_t ex = tp_block_scan<kBkThr>(cnt, lds, &tot) + carry;
    if (j < D) {
      const uint32_t slot = (uint32_t)v & 0xffffu;
      const int64_t u = (int64_t)ubase + j;
      if (in_range(u, u_cap)) {
        uniq[u] = key0 | (uint32_t)(v >> 32);
        seg_start[u] = (int32_t)(ebase + ex);
        if (zero_a) zero_a[u] = 0.f;
        if (zero_b) zero_b[u] = 0ull;
      }
      cur[slot] = ex;
      jj[slot] = (uint16_t)j;
    }
    carry += tot;
  }
  __syncthreads();
  if (prof && t == 0) prof[(int64_t)blockIdx.x * 12 + 6] = clock64();
#pragma unroll
  for (int q = 0; q < kG; ++q) {
    if (idx[q] < 0) continue;
    const uint32_t h = eh[q * kBkThr + t];
    if (h == 0xffffu) continue;
    const uint32_t pos = atomicAdd(&cur[h], 1u);
    const uint32_t u = ubase + jj[h];
    const int64_t e = (int64_t)ebase + pos;
    if (in_range(e, e_cap)) {
      pos_s[e] = idx[q];
      segid[e] = (int32_t)(u + 1);
    }
    if (in_range((int64_t)idx[q], e_cap)) ent_uid[idx[q]] = (int32_t)u;
  }
  __syncthreads();
}

// Decoupled look-back of fine bucket fs (wave 0; the caller syncs after): the bases
// (sums of every earlier fine bucket's counts) go to sb[1] / sb[2]; the inclusive prefix
// is published at fs and at twin (a pair's second fine bucket, published empty); the
// workgroup holding the last fine bucket writes the totals and advances the epoch.
__device__ __forceinline__ void tp_bk_lookback(uint64_t* __restrict__ status, int fs, int twin,
                                               int nbf, uint32_t ep, uint32_t D, uint32_t E,
                                               uint32_t* sb, uint32_t* __restrict__ epoch,
                                               int32_t* __restrict__ n_uniq,
                                               int32_t* __restrict__ n_ent,
                                               int32_t* __restrict__ seg_start, int64_t u_cap,
                                               int32_t* __restrict__ err) {
  using namespace tp;
  const int lane = threadIdx.x;
  if (lane >= 64) return;
  uint32_t su = 0, se = 0;
  if (fs > 0) {
    int j = fs - 1;
    uint32_t spins = 0;
    while (true) {
      const int jl = j - lane;  // lane 0 = nearest earlier bucket
      const uint64_t st =
          jl >= 0 ? __hip_atomic_load(&status[jl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                  : tp_status(ep, kStP, 0, 0);
      const uint32_t f = (uint32_t)(st >> 56) == ep ? (uint32_t)(st >> 54) & 3u : 0u;
      const uint64_t pm = __ballot(f == kStP), nr = __ballot(f == 0);
      const int fp = pm ? __builtin_ctzll(pm) : 64;  // nearest inclusive prefix
      const uint64_t need = fp >= 63 ? ~0ull : ((2ull << fp) - 1);
      if (nr & need) {  // an earlier bucket has not published yet
        if (++spins > (1u << 22)) {
          if (lane == 0) atomicOr(err, 4);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      const bool inc = lane <= fp;
      su += wave_allsum(inc ? (uint32_t)(st >> 27) & kStM : 0u);
      se += wave_allsum(inc ? (uint32_t)st & kStM : 0u);
      if (fp < 64) break;
      j -= 64;
    }
  }
  if (lane == 0) {
    const uint64_t inc = tp_status(ep, kStP, su + D, se + E);
    if (fs > 0) __hip_atomic_store(&status[fs], inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (twin != fs) __hip_atomic_store(&status[twin], inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sb[1] = su;
    sb[2] = se;
    if (twin == nbf - 1) {  // every bucket has published: the launch is done with the epoch
      const uint32_t U = su + D, Et = se + E;
      *n_uniq = (int32_t)U;
      *n_ent = (int32_t)Et;
      if (in_range((int64_t)U, u_cap + 1)) seg_start[U] = (int32_t)Et;
      __hip_atomic_store(epoch, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Fallback for one fine bucket f of an overflowing pair, register-light (plain loops,
// no per-thread entry arrays, so it does not raise the common path's register count):
// the per-tile runs live in the eh region, entries are located again for the assign
// and find their key's rank by binary search in the sorted list.
__device__ __forceinline__ void tp_bk_fine_light(
    const uint32_t* __restrict__ tkeys, const uint16_t* __restrict__ toff, int nbf, int T,
    int shift, int f, uint32_t hb, uint64_t key0, uint32_t* hkey, uint32_t* hcnt, uint64_t* hs,
    uint64_t* dl, uint16_t* ehraw, uint32_t* lds, uint32_t* sb, uint64_t* __restrict__ status,
    uint32_t ep, uint32_t* __restrict__ epoch, int32_t* __restrict__ pos_s,
    int32_t* __restrict__ segid, uint64_t* __restrict__ uniq, int32_t* __restrict__ seg_start,
    int32_t* __restrict__ ent_uid, int32_t* __restrict__ n_uniq, int32_t* __restrict__ n_ent,
    float* __restrict__ zero_a, unsigned long long* __restrict__ zero_b, int64_t u_cap,
    int64_t e_cap, int32_t* __restrict__ err) {
  using namespace tp;
  static_assert((kMaxT + 1) * 4 + kMaxT * 2 <= kECapL * 2, "tile runs must fit in eh");
  const int t = threadIdx.x;
  uint32_t* tpre = reinterpret_cast<uint32_t*>(ehraw);             // [kMaxT + 1]
  uint16_t* tlo = reinterpret_cast<uint16_t*>(tpre + kMaxT + 1);  // [kMaxT]
  for (int s = t; s < kDH; s += kBkThr) {
    hkey[s] = kEmpty;
    hcnt[s] = 0;
  }
  const int per = (T + kBkThr - 1) / kBkThr;
  const int q0 = t * per, q1 = q0 + per < T ? q0 + per : T;
  uint32_t c = 0;
  for (int q = q0; q < q1; ++q) {
    const uint16_t* to = toff + (int64_t)q * (nbf + 1);
    const uint32_t lo = to[f], hi = to[f + 1];
    tlo[q] = (uint16_t)lo;
    tpre[q] = hi - lo;
    c += hi - lo;
  }
  uint32_t E;
  uint32_t w = tp_block_scan<kBkThr>(c, lds, &E);
  for (int q = q0; q < q1; ++q) {
    const uint32_t len = tpre[q];
    tpre[q] = w;
    w += len;
  }
  if (t == 0) tpre[T] = E;
  __syncthreads();
  auto locate = [&](uint32_t g) -> int32_t {
    int lo = 0, up = T - 1;  // last tile with tpre[q] <= g
    while (lo < up) {
      const int mid = (lo + up + 1) >> 1;
      if (tpre[mid] <= g) lo = mid; else up = mid - 1;
    }
    return lo * kTile + tlo[lo] + (int32_t)(g - tpre[lo]);
  };
  bool bad = false;
  for (uint32_t g = t; g < E; g += kBkThr) {
    const uint32_t key = tkeys[locate(g)] | (hb << shift);
    uint32_t h = tp_hash(key) & (kDH - 1);
    bool ok = false;
    // (bounded chain: a hash this full -- near-distinct keys -- is cheaper to give up on
    // than to probe through: the overflow form takes the pair, profiles/r6_skew_layout.log)
    for (int p = 0; p < kBkProbe && !bad; ++p) {
      const uint32_t cu = hkey[h];
      if (cu == kEmpty) {
        const uint32_t prev = atomicCAS(&hkey[h], kEmpty, key);
        if (prev == kEmpty || prev == key) { ok = true; break; }
      } else if (cu == key) {
        ok = true;
        break;
      }
      h = (h + 1) & (kDH - 1);
    }
    if (ok) atomicAdd(&hcnt[h], 1u);
    else bad = true;
  }
  if (bad) atomicOr(err, 1);
  __syncthreads();
  constexpr int kPer = kDH / kBkThr;
  uint32_t cc = 0;
  for (int q = 0; q < kPer; ++q) cc += hkey[q * kBkThr + t] != kEmpty;
  uint32_t D;
  uint32_t wd = tp_block_scan<kBkThr>(cc, lds, &D);
  for (int q = 0; q < kPer; ++q) {
    const int s = q * kBkThr + t;
    if (hkey[s] != kEmpty) dl[wd++] = ((uint64_t)hkey[s] << 32) | ((uint64_t)hcnt[s] << 16) | (uint64_t)s;
  }
  if (t == 0)
    __hip_atomic_store(&status[f], tp_status(ep, f == 0 ? kStP : kStA, D, E), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  tp_bk_ranksort(dl, hs, D);
  tp_bk_lookback(status, f, f, nbf, ep, D, E, sb, epoch, n_uniq, n_ent, seg_start, u_cap, err);
  __syncthreads();
  const uint32_t ubase = sb[1], ebase = sb[2];
  uint32_t* cur = reinterpret_cast<uint32_t*>(dl);  // [D] per sorted key
  uint32_t carry = 0;
  for (uint32_t j0 = 0; j0 < D; j0 += kBkThr) {
    const uint32_t j = j0 + t;
    const uint64_t v = j < D ? hs[j] : 0ull;
    const uint32_t cnt = (uint32_t)(v >> 16) & 0xffffu;
    uint32_t tot;
    const uint32_t ex = tp_block_scan<kBkThr>(cnt, lds, &tot) + carry;
    if (j < D) {
      const int64_t u = (int64_t)ubase + j;
      if (in_range(u, u_cap)) {
        uniq[u] = key0 | (uint32_t)(v >> 32);
        seg_start[u] = (int32_t)(ebase + ex);
        if (zero_a) zero_a[u] = 0.f;
        if (zero_b) zero_b[u] = 0ull;
      }
      cur[j] = ex;
    }
    carry += tot;
  }
  __syncthreads();
  for (uint32_t g = t; g < E; g += kBkThr) {
    const int32_t id = locate(g);
    const uint32_t key = tkeys[id] | (hb << shift);
    uint32_t lo = 0, up = D - 1;  // the sorted key's index
    while (lo < up) {
      const uint32_t mid = (lo + up) >> 1;
      if ((uint32_t)(hs[mid] >> 32) < key) lo = mid + 1; else up = mid;
    }
    if (D == 0 || (uint32_t)(hs[lo] >> 32) != key) continue;  // (only after an overflow)
    const uint32_t pos = atomicAdd(&cur[lo], 1u);
    const uint32_t u = ubase + lo;
    const int64_t e = (int64_t)ebase + pos;
    if (in_range(e, e_cap)) {
      pos_s[e] = id;
      segid[e] = (int32_t)(u + 1);
    }
    if (in_range((int64_t)id, e_cap)) ent_uid[id] = (int32_t)u;
  }
  __syncthreads();
}

// One workgroup per pair of fine buckets (pair = false: per fine bucket). The status
// words are per FINE bucket: a pair publishes its counts at 2b and an empty aggregate at
// 2b+1, so the look-back sums the same either way. A pair that overflows the LDS
// capacity or its hash (nearly distinct keys) processes its two fine buckets one after
// the other instead (tp_bk_fine_light), each with its own publish and look-back; the
// fine geometry keeps that exact even when every key is distinct. (Tried and dropped:
// redoing the whole launch in a gated fine-bucket kernel, +4.8 us per step for the
// empty launch; the fallback as a second copy of the register-staged path, 95 VGPRs.)
// (8 waves per SIMD = 4 workgroups per CU: <= 64 VGPRs)
__global__ void __launch_bounds__(tp::kBkThr, 8)
tp_bucket_kernel(const uint32_t* __restrict__ tkeys, const uint16_t* __restrict__ toff, int nbf,
                 int pair, int T, int shift, uint64_t* __restrict__ status,
                 uint32_t* __restrict__ epoch, int32_t* __restrict__ pos_s,
                 int32_t* __restrict__ segid, uint64_t* __restrict__ uniq,
                 int32_t* __restrict__ seg_start, int32_t* __restrict__ ent_uid,
                 int32_t* __restrict__ n_uniq, int32_t* __restrict__ n_ent,
                 float* __restrict__ zero_a, unsigned long long* __restrict__ zero_b,
                 int64_t u_cap, int64_t e_cap, int32_t* __restrict__ err,
                 uint64_t* __restrict__ prof) {
  using namespace tp;
  // 40,960 B of LDS (<= 40 KB: 4 workgroups of 512 threads per CU)
  __shared__ uint16_t eh[kECapL];   // hash slot of every gathered entry
  __shared__ uint64_t hs[kDH];      // hash (key u32 | count u32), then the sorted list
  __shared__ uint64_t dl[kDH];      // per-tile runs (until the inserts), then compacted
                                    // (key | count << 16 | slot), then cur/jj
  __shared__ uint32_t lds[kBkThr / 64 + 1];
  __shared__ uint32_t sb[4];        // epoch, unique base, entry base, build flag
  static_assert((kMaxT + 1) * 4 + kMaxT * 4 <= kDH * 8, "tile runs must fit in dl");
  uint32_t* hkey = reinterpret_cast<uint32_t*>(hs);
  uint32_t* hcnt = hkey + kDH;
  const int t = threadIdx.x, b = blockIdx.x;
  if (prof && t == 0) {
    prof[(int64_t)b * 12 + 0] = clock64();
    prof[(int64_t)b * 12 + 8] = __builtin_amdgcn_s_memrealtime();
  }
  if (t == 0) {
    uint32_t ep = (__hip_atomic_load(epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u) & 0xffu;
    sb[0] = ep ? ep : 1u;
  }
  const int f0 = pair ? 2 * b : b, twin = pair ? f0 + 1 : f0;
  const uint64_t key0 = (uint64_t)f0 << shift;
  int32_t idx[kG];
  uint32_t E, D;
  const bool good = tp_bk_build(tkeys, toff, nbf, T, shift, f0, pair ? 2 : 1, 0u, hkey, hcnt, dl,
                                eh, lds, &sb[3], idx, &E, &D, prof);
  const uint32_t ep = sb[0];
  if (!good && pair) {
#pragma unroll 1
    for (int s = 0; s < 2; ++s)
      tp_bk_fine_light(tkeys, toff, nbf, T, shift, f0 + s, (uint32_t)s, key0, hkey, hcnt, hs, dl,
                       eh, lds, sb, status, ep, epoch, pos_s, segid, uniq, seg_start, ent_uid,
                       n_uniq, n_ent, zero_a, zero_b, u_cap, e_cap, err);
    return;
  }
  if (!good && t == 0) atomicOr(err, 1);
  if (t == 0) {  // publish (fine bucket 0: its inclusive prefix); a pair's twin is empty
    if (twin != f0)
      __hip_atomic_store(&status[twin], tp_status(ep, kStA, 0, 0), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&status[f0], tp_status(ep, f0 == 0 ? kStP : kStA, D, E), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  if (prof && t == 0) prof[(int64_t)b * 12 + 3] = clock64();
  tp_bk_ranksort(dl, hs, D);
  if (prof && t == 0) prof[(int64_t)b * 12 + 4] = clock64();
  tp_bk_lookback(status, f0, twin, nbf, ep, D, E, sb, epoch, n_uniq, n_ent, seg_start, u_cap, err);
  __syncthreads();
  if (prof && t == 0) prof[(int64_t)b * 12 + 5] = clock64();
  tp_bk_emit(hs, dl, eh, idx, D, sb[1], sb[2], key0, lds, pos_s, segid, uniq, seg_start, ent_uid,
             zero_a, zero_b, u_cap, e_cap, prof);
  if (prof && t == 0) {
    prof[(int64_t)b * 12 + 7] = clock64();
    prof[(int64_t)b * 12 + 9] = __builtin_amdgcn_s_memrealtime();
  }
}

// ---------------------------------------------------------------------- gather
__global__ void tp_gather_kernel(const uint16_t* __restrict__ rep,
                                 const int32_t* __restrict__ ent_uid, int64_t n,
                                 int32_t* __restrict__ local_col) {
  constexpr int kPer = 4;
  const int64_t i0 = (blockIdx.x * (int64_t)blockDim.x) * kPer + threadIdx.x;
  int64_t e[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int64_t i = i0 + q * blockDim.x;
    e[q] = i < n ? (i / tp::kTile) * tp::kTile + rep[i] : -1;
  }
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int64_t i = i0 + q * blockDim.x;
    if (e[q] >= 0) local_col[i] = ent_uid[e[q]];
  }
}

// -------------------------------------------------------------------- backward
// psum[tile entry] = sum over the tile's occurrences of the entry of coef[row] * val.
// Tiles accumulate in 64-bit FIXED POINT with integer LDS atomics (gfx950: ds_add_f32
// ~195 cycles per wave-instruction, ds_add_u64 ~13-18; profiles/r2_lds_atomics.log):
// scale 2^(48 - e) with every |addend| < 2^e keeps any sum of a tile's 8192 addends
// below 2^61, and the partials are exactly rounded, order-independent sums.
__device__ __forceinline__ int fx_shift(uint32_t maxbits) {
  int e = 0;
  if (maxbits) (void)frexpf(__uint_as_float(maxbits), &e);
  return min(100, 48 - e);
}
__device__ __forceinline__ void fx_add(long long* acc, int idx, float v, double sc) {
  const long long fx = __double2ll_rn((double)v * sc);
  if (fx) atomicAdd(reinterpret_cast<unsigned long long*>(&acc[idx]), (unsigned long long)fx);
}
// every wave's max |v| -> the tile's (LDS ds_max_u32 on the float bits of |v|)
__device__ __forceinline__ void fx_tile_max(float vmax, uint32_t* smax) {
  vmax = wave_max(vmax);
  if ((threadIdx.x & 63) == 0 && vmax > 0.f) atomicMax(smax, __float_as_uint(vmax));
}

// Variable-width rows (rows != null): one LDS atomic per occurrence.
__global__ void __launch_bounds__(tp::kThr)
tp_bwd_accum_kernel(const uint16_t* __restrict__ rep, const int32_t* __restrict__ dcnt, int64_t n,
                    const int32_t* __restrict__ rows, int width, const float* __restrict__ vals,
                    const float* __restrict__ coef, int64_t B, float* __restrict__ psum) {
  using namespace tp;
  __shared__ long long acc[kTile];
  __shared__ uint32_t smax;
  const int t = threadIdx.x;
  for (int i = t; i < kTile; i += kThr) acc[i] = 0ll;
  if (t == 0) smax = 0u;
  const int64_t base = (int64_t)blockIdx.x * kTile;
  float v[kIt];
  uint16_t e[kIt];
  float vmax = 0.f;
#pragma unroll
  for (int j = 0; j < kIt; ++j) {
    const int64_t i = base + j * kThr + t;
    v[j] = 0.f;
    e[j] = 0;
    if (i < n) {
      const int64_t r = rows ? (int64_t)rows[i] : (int64_t)((uint32_t)i / (uint32_t)width);
      e[j] = rep[i];
      if (in_range(r, B)) v[j] = coef[r] * (vals ? vals[i] : 1.f);
    }
    vmax = fmaxf(vmax, fabsf(v[j]));
  }
  __syncthreads();  // acc / smax zeroed
  fx_tile_max(vmax, &smax);
  __syncthreads();
  const int k2 = fx_shift(smax);
  const double sc = ldexp(1.0, k2);
#pragma unroll
  for (int j = 0; j < kIt; ++j)
    if (v[j] != 0.f) fx_add(acc, e[j], v[j], sc);
  __syncthreads();
  const int cnt = min(kTile, max(0, dcnt[blockIdx.x]));
  const double isc = ldexp(1.0, -k2);
  for (int i = t; i < cnt; i += kThr) psum[base + i] = (float)((double)acc[i] * isc);
}

// Fixed-width rows: thread = (slot, run of L consecutive rows) walks down its column,
// so a hot key of a slot repeats along the walk and is summed in a register until the
// key changes (one LDS atomic per run instead of per occurrence); the lanes of a wave
// hold adjacent slots of the same rows, so the rep / vals loads stay coalesced.
// (Row-major lanes: LDS atomic waits on hot entries dominated, SQ_WAIT_INST_LDS.)
__global__ void __launch_bounds__(tp::kThr)
tp_bwd_accum_cols_kernel(const uint16_t* __restrict__ rep, const int32_t* __restrict__ dcnt,
                         int64_t n, int width, const float* __restrict__ vals,
                         const float* __restrict__ coef, int64_t B, float* __restrict__ psum) {
  using namespace tp;
  __shared__ long long acc[kTile];
  __shared__ uint32_t smax;
  const int t = threadIdx.x;
  for (int i = t; i < kTile; i += kThr) acc[i] = 0ll;
  if (t == 0) smax = 0u;
  const int64_t base = (int64_t)blockIdx.x * kTile;
  const int64_t lim = n - base < kTile ? n - base : kTile;
  const int64_t r0 = base / width, r1 = (base + lim - 1) / width;
  const int nr = (int)(r1 - r0 + 1);
  const int L = (nr * width + kThr - 1) / kThr;  // rows per thread
  const int nseg = (nr + L - 1) / L;
  const int slot = t % width, seg = t / width;
  const int ra = seg * L, rb = ra + L < nr ? ra + L : nr;
  constexpr int kL = 16;  // rows a thread prefetches into registers before its walk
  const bool regs = seg < nseg && L <= kL;
  uint32_t ee[kL];
  float vv[kL];
  float vmax = 0.f;
  if (regs) {
#pragma unroll
    for (int q = 0; q < kL; ++q) {  // every load of the walk in flight at once
      const int rl = ra + q;
      const int64_t r = r0 + rl;
      const int64_t i = r * width + slot;
      const bool ok = q < L && rl < nr && i >= base && i < base + lim && in_range(r, B);
      ee[q] = ok ? (uint32_t)rep[i] : 0xffffffffu;
      vv[q] = ok ? coef[r] * (vals ? vals[i] : 1.f) : 0.f;
      vmax = fmaxf(vmax, fabsf(vv[q]));
    }
  } else if (seg < nseg) {  // long walks (width > 1024 / kL rows): a max pre-pass
    for (int rl = ra; rl < rb; ++rl) {
      const int64_t r = r0 + rl;
      const int64_t i = r * width + slot;
      if (i >= base && i < base + lim && in_range(r, B))
        vmax = fmaxf(vmax, fabsf(coef[r] * (vals ? vals[i] : 1.f)));
    }
  }
  __syncthreads();  // acc / smax zeroed
  fx_tile_max(vmax, &smax);
  __syncthreads();
  const int k2 = fx_shift(smax);
  const double sc = ldexp(1.0, k2);
  uint32_t cur = 0xffffffffu;
  float sum = 0.f;  // a run of equal keys down the column (<= L addends < 2^e each)
  if (regs) {
#pragma unroll
    for (int q = 0; q < kL; ++q) {
      if (ee[q] == 0xffffffffu) continue;
      if (ee[q] != cur) {
        if (cur != 0xffffffffu && sum != 0.f) fx_add(acc, cur, sum, sc);
        cur = ee[q];
        sum = vv[q];
      } else {
        sum += vv[q];
      }
    }
  } else if (seg < nseg) {
    for (int rl = ra; rl < rb; ++rl) {
      const int64_t r = r0 + rl;
      const int64_t i = r * width + slot;  // global position
      if (i < base || i >= base + lim || !in_range(r, B)) continue;
      const uint32_t e = rep[i];
      const float v = coef[r] * (vals ? vals[i] : 1.f);
      if (e != cur) {
        if (cur != 0xffffffffu && sum != 0.f) fx_add(acc, cur, sum, sc);
        cur = e;
        sum = v;
      } else {
        sum += v;
      }
    }
  }
  if (cur != 0xffffffffu && sum != 0.f) fx_add(acc, cur, sum, sc);
  __syncthreads();
  const int cnt = min(kTile, max(0, dcnt[blockIdx.x]));
  const double isc = ldexp(1.0, -k2);
  for (int i = t; i < cnt; i += kThr) psum[base + i] = (float)((double)acc[i] * isc);
}

__global__ void __launch_bounds__(256)
tp_seg_reduce_kernel(const int32_t* __restrict__ pos_s, const int32_t* __restrict__ segid,
                     int64_t n_host, const int32_t* __restrict__ n_dev,
                     const float* __restrict__ psum, int64_t p_cap, float* __restrict__ grad,
                     int64_t grad_cap) {
  // segmented scan over the entry CSC on DPP lane moves (no ds_bpermute); run ends
  // store grad[u], runs cut by a wave boundary add atomically (grad zeroed by emit)
  const int lane = threadIdx.x & 63;
  const int64_t n = dev_len(n_dev, n_host);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); i0 < n;
       i0 += stride) {
    const int64_t i = i0 + lane;
    const bool valid = i < n;
    int32_t s = -3;
    float x[1] = {0.f};
    if (valid) {
      s = segid[i];
      const int32_t p = pos_s[i];
      if (in_range(p, p_cap)) x[0] = psum[p];
    }
    const int32_t s_next = i + 1 < n ? segid[i + 1] : -1;
    const int32_t s_prev0 = i0 > 0 ? segid[i0 - 1] : -1;
    seg_scan_step<0x111, 0xf>(s, x);
    seg_scan_step<0x112, 0xf>(s, x);
    seg_scan_step<0x114, 0xf>(s, x);
    seg_scan_step<0x118, 0xf>(s, x);
    seg_scan_step<0x142, 0xa>(s, x);
    seg_scan_step<0x143, 0xc>(s, x);
    const int32_t s_lane0 = __builtin_amdgcn_readfirstlane(s);
    if (valid && (s_next != s || lane == 63)) {
      const bool starts_inside = s != s_lane0 || s_prev0 != s;
      const int32_t u = s - 1;
      if (in_range(u, grad_cap)) {
        if (starts_inside && s_next != s) grad[u] = x[0];
        else atomicAdd(&grad[u], x[0]);
      }
    }
  }
}

// Entry scan fused with the 1-GPU optimizer update (replaces tp_seg_reduce + kv_update:
// one launch and the grad[] round trip less). The segmented scan of tp_seg_reduce;
// a key whose entries all lie in one wave's 64-entry chunk has its full gradient in
// the lane that ends the run, which applies the update to the key's slot at once.
// A key spanning several chunks (hot keys: <= #tiles entries, so <= 6 chunks) adds
// each piece as ONE 64-bit integer atomic to acc[u] (zeroed by the bucket kernel):
// the piece in fixed point (scale 2^30) shifted left by 8, plus 1 in the low byte. The
// atomic returns the running (sum, count) together, so the piece that completes the
// count (chunks spanned, from seg_start) holds the whole sum and applies the update -
// no fence, no re-read (a device-scope __threadfence writes back the XCD's L2 and made
// a fence-based version 6x slower than the unfused pair). Binary features only (the
// host checks): |gradient| <= rows < 2^25 fits the 56-bit fixed-point field.
// Block 0 also turns the step's AUC histogram into metrics (as kv_update did).
__global__ void __launch_bounds__(256)
tp_seg_update_kernel(const int32_t* __restrict__ pos_s, const int32_t* __restrict__ segid,
                     int64_t n_host, const int32_t* __restrict__ n_dev,
                     const float* __restrict__ psum, int64_t p_cap,
                     const int32_t* __restrict__ seg_start, const int32_t* __restrict__ n_uniq,
                     unsigned long long* __restrict__ acc, int64_t u_cap,
                     const int64_t* __restrict__ slot_idx, Slot* __restrict__ slots, int64_t cap,
                     UpdateParams p, double* __restrict__ stats, int acc_stripes,
                     uint32_t* __restrict__ hist, int nbins, int hist_stripes,
                     double* __restrict__ metrics, int64_t* __restrict__ step_counter) {
  if (hist && blockIdx.x == 0) auc_hist_block(hist, nbins, hist_stripes, metrics, step_counter);
  const int lane = threadIdx.x & 63;
  const int64_t n = dev_len(n_dev, n_host);
  const int64_t U = dev_len(n_uniq, u_cap);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  double dnnz = 0, wsum = 0, dsum = 0;
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); i0 < n;
       i0 += stride) {
    const int64_t i = i0 + lane;
    const bool valid = i < n;
    int32_t s = -3;
    float x[1] = {0.f};
    if (valid) {
      s = segid[i];
      const int32_t q = pos_s[i];
      if (in_range(q, p_cap)) x[0] = psum[q];
    }
    const int32_t s_next = i + 1 < n ? segid[i + 1] : -1;
    const int32_t s_prev0 = i0 > 0 ? segid[i0 - 1] : -1;
    seg_scan_step<0x111, 0xf>(s, x);
    seg_scan_step<0x112, 0xf>(s, x);
    seg_scan_step<0x114, 0xf>(s, x);
    seg_scan_step<0x118, 0xf>(s, x);
    seg_scan_step<0x142, 0xa>(s, x);
    seg_scan_step<0x143, 0xc>(s, x);
    const int32_t s_lane0 = __builtin_amdgcn_readfirstlane(s);
    if (!(valid && (s_next != s || lane == 63))) continue;
    const int64_t u = (int64_t)s - 1;
    if (u < 0 || u >= U) continue;
    const bool starts_inside = s != s_lane0 || s_prev0 != s;
    float g = x[0];
    bool apply = starts_inside && s_next != s;
    if (!apply) {  // a piece of a key spanning several 64-entry chunks
      const long long fx = __double2ll_rn((double)g * 1073741824.0);  // 2^30
      const unsigned long long add = ((unsigned long long)fx << 8) + 1ull;
      const unsigned long long tot = atomicAdd(&acc[u], add) + add;
      const int64_t e0 = seg_start[u], e1 = seg_start[u + 1];
      const uint32_t np = (uint32_t)((e1 - 1) / 64 - e0 / 64 + 1);
      if ((uint32_t)(tot & 0xffull) == np) {
        g = (float)((double)((long long)tot >> 8) * (1.0 / 1073741824.0));
        apply = true;
      }
    }
    if (!apply) continue;
    const int64_t si = slot_idx[u];
    if (!in_range(si, cap)) continue;
    const float gs = g * p.grad_scale;
    if (gs != gs) continue;  // NaN mark = filtered entry
    Slot sl = slots[si];
    const float w_old = apply_update(sl, gs, p);
    slots[si] = sl;
    dnnz += (double)((sl.w != 0.f) - (w_old != 0.f));
    wsum += (double)sl.w * sl.w;
    const double d = (double)sl.w - w_old;
    dsum += d * d;
  }
  if (stats) {
    const double a = wave_sum_dpp(dnnz), b = wave_sum_dpp(wsum), c = wave_sum_dpp(dsum);
    if (lane == 63) {
      double* st = acc_stripe(stats, acc_stripes);
      if (a != 0) atomicAdd(&st[0], a);
      if (b != 0) atomicAdd(&st[1], b);
      if (c != 0) atomicAdd(&st[2], c);
    }
  }
}

// Fused forward + per-tile backward of a fixed-width linear model on a tp
// localisation, one workgroup per 8192-occurrence tile (replaces the local-column
// gather, linear_fwd and tp_bwd_accum: three launches and two global round trips).
// Every row overlapping the tile gets kFbLanes lanes strided over its occurrences.
//   prologue (all global loads in flight together): each lane's occurrences
//     (rep, val) into registers, the rows' labels into LDS, the tile's entry
//     weights wl[e] = w_local[ent_uid[tile + e]] into LDS; an occurrence of a row
//     cut by the tile boundary resolves its weight through the global entry map
//     and keeps w * val in its register slot;
//   forward: margins from registers + LDS, a DPP reduction per lane group, the
//     leader computes the loss terms (the tile holding a row's first occurrence
//     owns its coef output, metrics and AUC bin);
//   backward: the same registers add coef * val into per-entry accumulators at rep,
//     then the per-entry partials psum[tile + e] go to tp_seg_reduce_kernel.
// The backward accumulates in 64-bit FIXED POINT with integer LDS atomics: on gfx950 a
// ds_add_f32 wave-instruction costs ~195 cycles whatever the addresses, ds_add_u64
// ~13-18 (benchmarks/micro/lds_atomics.hip, profiles/r2_lds_atomics.log), and the
// float atomics were 45 % of the kernel. The tile's scale 2^k (k = 48 - e, every
// |coef * val| < 2^e) keeps any sum of 8192 addends below 2^61 and quantises each
// addend at 2^-(k+1) relative to the tile's largest: the partials are the exactly
// rounded sums, independent of atomic order (deterministic).
// PER = occurrences per lane per row (width <= 8 * PER), NP = row passes held in
// registers (128 rows each): compile-time so the register slots stay registers.
constexpr int kFbLanes = 8;
constexpr int kFbMaxRows = tp::kTile / 8 + 2;  // width >= 8
constexpr int kFbMaxBins = 2048;                // AUC bins held in LDS (2 x 2048 u32)
constexpr uint16_t kFbNone = 0xffff, kFbExt = 0xfffe;

// Sum over the 8 lanes of an aligned lane group, result in all 8 (DPP: quad_perm
// [1,0,3,2], [2,3,0,1], then row_half_mirror; no LDS crossbar, bitwise equal in all 8).
__device__ __forceinline__ float group8_sum(float m) {
  m += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(m), 0xB1, 0xf, 0xf, false));
  m += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(m), 0x4E, 0xf, 0xf, false));
  m += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(m), 0x141, 0xf, 0xf, false));
  return m;
}

// Phase marks of the fused kernel (a tuning aid, benchmarks/prof_tp_phases.py): null
// unless tp_fb_set_prof() installed a buffer of 16 u64 per workgroup.
__device__ uint64_t* g_fb_prof = nullptr;
#define FB_MARK(k)                                                             \
  if (fbp && threadIdx.x == 0) fbp[(int64_t)blockIdx.x * 16 + (k)] = clock64()

// kFlat (the flat 1-GPU path, tpf_step): w_local is already in tile-entry order
// (w_ent[tile * 8192 + e], scattered there by the step boundary kernel), so the
// prologue reads the tile's weights contiguously instead of the dependent
// ent_uid -> w_local gather (19 k of 37 k cycles per workgroup, r3_tp_pair_phases.log).
template <int PER, int NP, bool kFlat>
__global__ void __launch_bounds__(tp::kThr)  // 68 KB LDS -> 2 workgroups per CU
tp_fwd_bwd_kernel(const uint16_t* __restrict__ rep, const int32_t* __restrict__ dcnt,
                  const int32_t* __restrict__ ent_uid, int64_t n, int width,
                  const float* __restrict__ vals, const float* __restrict__ w_local, int64_t w_cap,
                  const float* __restrict__ labels, int64_t B, int loss_type,
                  float* __restrict__ coef_out, double* __restrict__ metrics,
                  uint32_t* __restrict__ hist, int nbins, int acc_stripes, int hist_stripes,
                  float* __restrict__ psum, int lts) {
  using namespace tp;
  // one 64 KB region: forward = entry weights (f32, [0, 32 KB)) + AUC histogram
  // ([32 KB, 48 KB)); backward = the entries' fixed-point accumulators (i64)
  __shared__ unsigned long long region[kTile];
  __shared__ float crow[kFbMaxRows];  // labels of the tile's rows
  __shared__ float sacc[4];           // tile sums of loss, correct, rows
  __shared__ uint32_t smax;           // bits of the tile's largest |coef * val|
  float* const wl = reinterpret_cast<float*>(region);
  uint32_t* const lhist = reinterpret_cast<uint32_t*>(region) + kTile;
  long long* const acc = reinterpret_cast<long long*>(region);
  constexpr int kRowsPass = kThr / kFbLanes;
  const int t = threadIdx.x, sub = t % kFbLanes, g = t / kFbLanes;
  // occurrences [base, base + lim) (2^lts per tile), entries [eb, eb + cnt)
  const int64_t base = (int64_t)blockIdx.x << lts, eb = (int64_t)blockIdx.x * kTile;
  const int lim = (int)(n - base < (1 << lts) ? n - base : (1 << lts));
  const int64_t r0 = base / width;
  const int nr = (int)((base + lim - 1) / width - r0 + 1);
  const int cnt = min(kTile, max(0, dcnt[blockIdx.x]));
  uint64_t* const fbp = g_fb_prof;
  if (fbp && threadIdx.x == 0) fbp[(int64_t)blockIdx.x * 16 + 8] = __builtin_amdgcn_s_memrealtime();
  FB_MARK(0);
  uint16_t ce[NP][PER];
  float cv[NP][PER];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int ri = p * kRowsPass + g;
    const int64_t r = r0 + ri;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int k = sub + q * kFbLanes;
      ce[p][q] = kFbNone;
      cv[p][q] = 0.f;
      if (ri < nr && r < B && k < width) {
        const int64_t i = r * width + k;
        const int64_t o = i - base;
        const bool in = o >= 0 && o < lim;
        const uint16_t e = rep[i];  // outside the tile: the entry in the neighbour tile
        ce[p][q] = in ? e : kFbExt;
        cv[p][q] = in ? (vals ? vals[i] : 1.f) : __int_as_float((int)e);
      }
    }
  }
  if (t < 4) sacc[t] = 0.f;
  if (t == 0) smax = 0u;
  // boundary rows: the outside part of row 0 / row nr-1 (only their lane groups) read
  // their weights through the neighbour tile's entry map; issued first, so the chain
  // rep -> ent_uid -> w_local overlaps the tile's own entry-weight loads
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int ri = p * kRowsPass + g;
    if (ri != 0 && ri != nr - 1) continue;
#pragma unroll
    for (int q = 0; q < PER; ++q)
      if (ce[p][q] == kFbExt) {
        const int64_t i = (r0 + ri) * width + sub + q * kFbLanes;
        const int64_t ge = (i >> lts) * kTile + __float_as_int(cv[p][q]);
        const int64_t u = kFlat ? ge : (int64_t)ent_uid[ge];
        cv[p][q] = (in_range(u, w_cap) ? w_local[u] : 0.f) * (vals ? vals[i] : 1.f);
      }
  }
  for (int i = t; i < nr; i += kThr) crow[i] = r0 + i < B ? labels[r0 + i] : 0.f;
  if (kFlat) {
    for (int i = t; i < cnt; i += kThr) wl[i] = w_local[eb + i];  // (host: w_cap >= T * 8192)
  } else {
    for (int i = t; i < cnt; i += kThr) {
      const int32_t u = ent_uid[eb + i];
      wl[i] = in_range(u, w_cap) ? w_local[u] : 0.f;
    }
  }
  if (hist)
    for (int i = t; i < 2 * nbins; i += kThr) lhist[i] = 0u;
  __syncthreads();
  FB_MARK(1);
  float loss_acc = 0.f, corr_acc = 0.f, rows_acc = 0.f;
  float cf[NP];
  float vmax = 0.f;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    float m = 0.f;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const uint16_t e = ce[p][q];
      if (e == kFbExt) m += cv[p][q];
      else if (e != kFbNone) m += wl[e] * cv[p][q];
    }
    m = group8_sum(m);
    const int ri = p * kRowsPass + g;
    const int64_t r = r0 + ri;
    float c = 0.f;
    if (ri < nr && r < B) {
      const float lab = crow[ri];
      float loss, c2;
      loss_terms(m, lab, loss_type, loss, c, c2);
      if (sub == 0 && r * width >= base) {  // first occurrence in this tile: the row is ours
        coef_out[r] = c;
        loss_acc += loss;
        corr_acc += ((lab > 0.f) == (m > 0.f)) ? 1.f : 0.f;
        rows_acc += 1.f;
        if (hist) atomicAdd(&lhist[auc_bin(m, lab, nbins)], 1u);
      }
    }
    cf[p] = c;  // every lane of the group holds its row's coef
#pragma unroll
    for (int q = 0; q < PER; ++q)
      if (ce[p][q] < kFbExt) vmax = fmaxf(vmax, fabsf(c * cv[p][q]));
  }
  fx_tile_max(vmax, &smax);
  if (metrics && rows_acc > 0.f) {  // leader lanes: tile sums (ds_add_f32, 3 per leader)
    atomicAdd(&sacc[0], loss_acc);
    atomicAdd(&sacc[1], corr_acc);
    atomicAdd(&sacc[2], rows_acc);
  }
  __syncthreads();
  FB_MARK(2);
  if (hist) {  // flush the AUC bins before the region turns into accumulators
    uint32_t* hs = hist + (int64_t)(blockIdx.x % hist_stripes) * 2 * nbins;
    for (int i = t; i < 2 * nbins; i += kThr)
      if (lhist[i]) atomicAdd(&hs[i], lhist[i]);
  }
  if (metrics && t == 0 && sacc[2] > 0.f) {
    double* mt = acc_stripe(metrics, acc_stripes);
    atomicAdd(&mt[0], (double)sacc[0]);
    atomicAdd(&mt[1], (double)sacc[1]);
    atomicAdd(&mt[2], (double)sacc[2]);
  }
  const uint32_t mb = smax;
  __syncthreads();
  for (int i = t; i < cnt; i += kThr) acc[i] = 0ll;
  __syncthreads();
  FB_MARK(3);
  const int k2 = fx_shift(mb);  // every |addend| < 2^e -> scale 2^(48 - e)
  const double sc = ldexp(1.0, k2);
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    if (cf[p] == 0.f) continue;
#pragma unroll
    for (int q = 0; q < PER; ++q)
      if (ce[p][q] < kFbExt) fx_add(acc, ce[p][q], cf[p] * cv[p][q], sc);  // ds_add_u64
  }
  FB_MARK(4);
  __syncthreads();
  FB_MARK(5);
  const double isc = ldexp(1.0, -k2);
  for (int i = t; i < cnt; i += kThr) psum[eb + i] = (float)((double)acc[i] * isc);
  FB_MARK(6);
  if (fbp && threadIdx.x == 0) {
    fbp[(int64_t)blockIdx.x * 16 + 9] = __builtin_amdgcn_s_memrealtime();
    fbp[(int64_t)blockIdx.x * 16 + 10] = __smid();
  }
}
#undef FB_MARK

// Variable-width / valued rows (CSR ``row_ptr`` + per-occurrence ``rows``, optional
// ``vals``; reference SparseMatrix::rangeTimes, src/util/sparse_matrix.h:73-107): the
// same fused forward + tile backward per 8192-occurrence tile as tp_fwd_bwd_kernel, for
// rows of any width. Thread t holds the tile's occurrences [8t, 8t+8) in registers
// (entry, value, row); a row's margin is summed in registers along the thread's run and
// added into an LDS row array once per run (rows of the tile: <= kCsrRows per window,
// windows repeat for tiles of very short rows). A row that starts before the tile or
// ends after it (the boundary rows) gets its outside part from one wave each, through
// the neighbour tiles' entry maps (flat: w_ent in tile-entry order). Every tile that
// holds part of a row computes that row's margin in full, so each uses the row's coef
// for its own entries; only the tile holding the row's first occurrence reports it
// (coef_out, loss, accuracy, AUC bin). Backward: 64-bit fixed point per tile entry
// (scale from the tile's largest |coef x val|), as the fixed-width kernel.
constexpr int kCsrRows = 4080;  // LDS row slots of one window (80 KB of LDS in all: 2 per CU)
// (~90 VGPRs: one workgroup per CU; a 64-VGPR bound spilled 100 B per lane. Real-data
// minibatches of this path are 10-600 tiles, so the grid rarely fills 2 per CU anyway.)
template <bool kFlat>
__global__ void __launch_bounds__(tp::kThr)
tp_fwd_bwd_csr_kernel(const uint16_t* __restrict__ rep, const int32_t* __restrict__ dcnt,
                      const int32_t* __restrict__ ent_uid, int64_t n,
                      const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ rows,
                      const float* __restrict__ vals, const float* __restrict__ w_local,
                      int64_t w_cap, const float* __restrict__ labels, int64_t B, int loss_type,
                      float* __restrict__ coef_out, double* __restrict__ metrics,
                      uint32_t* __restrict__ hist, int nbins, int acc_stripes, int hist_stripes,
                      float* __restrict__ psum, int lts) {
  using namespace tp;
  __shared__ unsigned long long region[kTile];  // fwd: entry weights + AUC bins; bwd: i64 acc
  __shared__ float crow[kCsrRows];              // a window's row margins, then their coefs
  __shared__ float sacc[4];
  __shared__ float sc0;                         // coef of row r0 when an earlier tile owns it
  __shared__ uint32_t smax;
  float* const wl = reinterpret_cast<float*>(region);
  uint32_t* const lhist = reinterpret_cast<uint32_t*>(region) + kTile;
  long long* const acc = reinterpret_cast<long long*>(region);
  constexpr int kPer = kTile / kThr;  // 8 occurrences per thread
  constexpr uint32_t kNone = 0xffffffffu;
  const int t = threadIdx.x;
  // occurrences [base, base + lim) (2^lts per tile), entries [eb, eb + cnt)
  const int64_t base = (int64_t)blockIdx.x << lts, eb = (int64_t)blockIdx.x * kTile;
  const int lim = (int)(n - base < (1 << lts) ? n - base : (1 << lts));
  const int cnt = min(kTile, max(0, dcnt[blockIdx.x]));
  const int64_t r0 = rows[base], r1 = rows[base + lim - 1];  // (uniform loads)
  // occurrence = (row - r0) << 13 | tile entry (entries < 2^13; a tile's row span, empty
  // rows included, < 2^19 - 1: the host routes B >= kCsrMaxRows elsewhere)
  uint32_t er[kPer];
  float v[kPer];
  {  // 8 consecutive occurrences per thread: 16 / 32-byte loads, adjacent across lanes
    const int64_t i0 = base + (int64_t)t * kPer;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const bool in = t * kPer + j < lim;
      const int64_t i = in ? i0 + j : base;
      const uint32_t ee = rep[i];
      const int32_t rr = rows[i];
      er[j] = in ? (uint32_t)(rr - r0) << 13 | ee : kNone;
      v[j] = in ? (vals ? vals[i] : 1.f) : 0.f;
    }
  }
  const bool own0 = row_ptr[r0] >= base;
  if (t < 4) sacc[t] = 0.f;
  if (t == 0) smax = 0u;
  if (kFlat) {
    for (int i = t; i < cnt; i += kThr) wl[i] = w_local[eb + i];
  } else {
    for (int i = t; i < cnt; i += kThr) {
      const int32_t u = ent_uid[eb + i];
      wl[i] = in_range(u, w_cap) ? w_local[u] : 0.f;
    }
  }
  if (hist)
    for (int i = t; i < 2 * nbins; i += kThr) lhist[i] = 0u;
  const int wave = t / 64, lane = t % 64;
  const int nr = (int)(r1 - r0 + 1);
  float loss_acc = 0.f, corr_acc = 0.f, rows_acc = 0.f;
  for (int wa = 0; wa < nr; wa += kCsrRows) {  // row windows (1 unless rows are tiny)
    const int wb = min(nr, wa + kCsrRows);
    for (int i = t; i < wb - wa; i += kThr) crow[i] = 0.f;
    __syncthreads();
    {  // this thread's runs of equal rows -> one LDS add per run
      uint32_t cur = kNone;
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        if (er[j] == kNone) continue;
        const uint32_t rr = er[j] >> 13;
        if (rr != cur) {
          if (cur != kNone && (int)cur >= wa && (int)cur < wb && sum != 0.f)
            atomicAdd(&crow[cur - wa], sum);
          cur = rr;
          sum = 0.f;
        }
        sum += wl[er[j] & 0x1fffu] * v[j];
      }
      if (cur != kNone && (int)cur >= wa && (int)cur < wb && sum != 0.f)
        atomicAdd(&crow[cur - wa], sum);
    }
    // boundary rows: wave 0 sums the part of row r0 before the tile, wave 1 the part of
    // row r1 after it (any length; a row longer than a tile has both)
    if (wave < 2) {
      const int rl = wave == 0 ? 0 : nr - 1;
      if (rl >= wa && rl < wb) {
        const int64_t r = r0 + rl;
        const int64_t a = wave == 0 ? row_ptr[r] : base + lim;
        const int64_t b = wave == 0 ? base : row_ptr[r + 1];
        float sum = 0.f;
        for (int64_t i = a + lane; i < b; i += 64) {
          const int64_t ge = (i >> lts) * kTile + (int64_t)rep[i];
          const int64_t u = kFlat ? ge : (int64_t)ent_uid[ge];
          sum += (in_range(u, w_cap) ? w_local[u] : 0.f) * (vals ? vals[i] : 1.f);
        }
        sum = wave_sum(sum);
        if (lane == 0 && sum != 0.f) atomicAdd(&crow[rl - wa], sum);
      }
    }
    __syncthreads();
    for (int i = t; i < wb - wa; i += kThr) {  // per row: loss terms -> coef
      const int64_t r = r0 + wa + i;
      float c = 0.f;
      if (r < B) {
        const float m = crow[i];
        const float lab = labels[r];
        float loss, c2;
        loss_terms(m, lab, loss_type, loss, c, c2);
        if (wa + i > 0 || own0) {  // the row's first occurrence is in this tile
          coef_out[r] = c;
          loss_acc += loss;
          corr_acc += ((lab > 0.f) == (m > 0.f)) ? 1.f : 0.f;
          rows_acc += 1.f;
          if (hist) atomicAdd(&lhist[auc_bin(m, lab, nbins)], 1u);
        } else {
          sc0 = c;
        }
      }
      crow[i] = c;
    }
    __syncthreads();
  }
  {  // empty rows (no occurrence) outside every tile's [first row, last row]: the gap
     // between the previous tile's last row and this tile's first (tile 0: from row 0)
     // and, in the last tile, the rows after its last one. Margin 0.
    const int64_t g0 = blockIdx.x == 0 ? 0 : (int64_t)rows[base - 1] + 1;
    const int64_t na = r0 > g0 ? r0 - g0 : 0;  // [g0, r0) (none when a row spans the cut)
    const int64_t nb = base + lim >= n && B > r1 + 1 ? B - (r1 + 1) : 0;  // (r1, B)
    for (int64_t i = t; i < na + nb; i += kThr) {
      const int64_t rr = i < na ? g0 + i : r1 + 1 + (i - na);
      const float lab = labels[rr];
      float loss, c, c2;
      loss_terms(0.f, lab, loss_type, loss, c, c2);
      coef_out[rr] = c;
      loss_acc += loss;
      corr_acc += (lab > 0.f) == false ? 1.f : 0.f;
      rows_acc += 1.f;
      if (hist) atomicAdd(&lhist[auc_bin(0.f, lab, nbins)], 1u);
    }
  }
  // coef of an occurrence's row: the window in LDS (one window), else the row's coef as
  // this workgroup wrote it to coef_out (sc0 for a row an earlier tile owns)
  const bool one = nr <= kCsrRows;
  auto coef_of = [&](uint32_t rr) -> float {
    if (one) return crow[rr];
    if (rr == 0 && !own0) return sc0;
    return coef_out[r0 + rr];
  };
  float vmax = 0.f;
#pragma unroll
  for (int j = 0; j < kPer; ++j)
    if (er[j] != kNone) vmax = fmaxf(vmax, fabsf(coef_of(er[j] >> 13) * v[j]));
  fx_tile_max(vmax, &smax);
  if (metrics && rows_acc > 0.f) {
    atomicAdd(&sacc[0], loss_acc);
    atomicAdd(&sacc[1], corr_acc);
    atomicAdd(&sacc[2], rows_acc);
  }
  __syncthreads();
  if (hist) {
    uint32_t* hs = hist + (int64_t)(blockIdx.x % hist_stripes) * 2 * nbins;
    for (int i = t; i < 2 * nbins; i += kThr)
      if (lhist[i]) atomicAdd(&hs[i], lhist[i]);
  }
  if (metrics && t == 0 && sacc[2] > 0.f) {
    double* mt = acc_stripe(metrics, acc_stripes);
    atomicAdd(&mt[0], (double)sacc[0]);
    atomicAdd(&mt[1], (double)sacc[1]);
    atomicAdd(&mt[2], (double)sacc[2]);
  }
  const uint32_t mb = smax;
  __syncthreads();
  for (int i = t; i < cnt; i += kThr) acc[i] = 0ll;
  __syncthreads();
  const int k2 = fx_shift(mb);
  const double sc = ldexp(1.0, k2);
#pragma unroll
  for (int j = 0; j < kPer; ++j)
    if (er[j] != kNone) {
      const float c = coef_of(er[j] >> 13);
      if (c != 0.f) fx_add(acc, er[j] & 0x1fffu, c * v[j], sc);
    }
  __syncthreads();
  const double isc = ldexp(1.0, -k2);
  for (int i = t; i < cnt; i += kThr) psum[eb + i] = (float)((double)acc[i] * isc);
}

void tp_fb_set_prof(uint64_t* p) {
  PSAMD_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_fb_prof), &p, sizeof(p)));
}

// ====================================================================== flat ("tpf")
// The 1-GPU layout: the bucket stage writes FIXED per-workgroup output regions instead of
// one compact sorted array, so no bucket waits for another (the compact layout's
// decoupled look-back: 11 k of 47 k cycles per workgroup, r3_tp_pair_phases.log) and
// nothing is rank-sorted or laid out as a CSC. Bucket workgroup b (a pair of fine
// buckets, the tp_bucket geometry) owns
//   keys     uniqf[b * kUC + s * kUnitK + j], j < D_s   (unit s = 0; units 0 and 1 when an
//            overflowing pair falls back to its two fine buckets one after the other)
//   entries  ent_pos / ent_j[b * kEC + e]: tile entry id (tile * 8192 + e) and the unit's
//            key index j of every tile-distinct entry of the unit's keys (unit 1 after
//            the E_0 entries of unit 0)
//   counts   cnt[b * 4 + {D_0, E_0, D_1, E_1}]
// The consumers run one workgroup per bucket workgroup and combine in LDS: tpf_step sums
// each key's entry partials (fixed point) and applies the update, then pulls the next
// minibatch's keys and scatters their weights into its tile-entry order (w_ent), which
// the fused forward reads contiguously. Keys of one key-range bucket stay in the same
// bucket workgroup for every minibatch of the same size, so a key's update and its next
// pull run in the same workgroup, in that order.
namespace tpf {
constexpr int kUnitK = tp::kDH;  // keys of one unit (the bucket hash)
constexpr int kUC = 2 * kUnitK;  // key region of a bucket workgroup (two units)
constexpr int kEC = 8192;        // entry region of a bucket workgroup
constexpr int kThr = 256;        // tpf_step workgroup (auc_hist_block: an extra last one)
constexpr uint32_t kNoSlot = 0xffffffffu;
}  // namespace tpf

// Overflow unit (an overflowing pair's fine bucket f, or a lone bucket whose entries
// exceed the LDS capacity): register-light like tp_bk_fine_light; entries are located
// again from the per-tile runs for every pass, their key index found by probing the hash.
// Writes D / E into co[0..1] and returns E (block-uniform, via lds).
__device__ __forceinline__ uint32_t tpf_unit_light(
    const uint32_t* __restrict__ tkeys, const uint16_t* __restrict__ toff, int nbf, int T,
    int shift, int f, uint32_t hb, uint64_t key0, uint32_t* hkey, uint32_t* hmap,
    uint16_t* ehraw, uint32_t* lds, uint64_t* __restrict__ uo, int32_t* __restrict__ po,
    uint16_t* __restrict__ jo, uint32_t eoff, int32_t* __restrict__ co,
    int32_t* __restrict__ err, bool sorted) {
  using namespace tp;
  const int t = threadIdx.x;
  uint32_t* tpre = reinterpret_cast<uint32_t*>(ehraw);             // [kMaxT + 1]
  uint16_t* tlo = reinterpret_cast<uint16_t*>(tpre + kMaxT + 1);  // [kMaxT]
  for (int s = t; s < kDH; s += kBkThr) hkey[s] = kEmpty;
  const int per = (T + kBkThr - 1) / kBkThr;
  const int q0 = t * per, q1 = q0 + per < T ? q0 + per : T;
  uint32_t c = 0;
  for (int q = q0; q < q1; ++q) {
    const uint16_t* to = toff + (int64_t)q * (nbf + 1);
    const uint32_t lo = to[f], hi = to[f + 1];
    tlo[q] = (uint16_t)lo;
    tpre[q] = hi - lo;
    c += hi - lo;
  }
  uint32_t E;
  uint32_t w = tp_block_scan<kBkThr>(c, lds, &E);
  for (int q = q0; q < q1; ++q) {
    const uint32_t len = tpre[q];
    tpre[q] = w;
    w += len;
  }
  if (t == 0) tpre[T] = E;
  __syncthreads();
  auto locate = [&](uint32_t g) -> int32_t {
    int lo = 0, up = T - 1;  // last tile with tpre[q] <= g
    while (lo < up) {
      const int mid = (lo + up + 1) >> 1;
      if (tpre[mid] <= g) lo = mid; else up = mid - 1;
    }
    return lo * kTile + tlo[lo] + (int32_t)(g - tpre[lo]);
  };
  // probe (insert = true: claim an empty slot); returns the slot or -1
  auto probe = [&](uint32_t key, bool insert) -> int {
    uint32_t h = tp_hash(key) & (kDH - 1);
    for (int p = 0; p < kDH; ++p) {
      const uint32_t cu = hkey[h];
      if (cu == key) return (int)h;
      if (cu == kEmpty) {
        if (!insert) return -1;
        const uint32_t prev = atomicCAS(&hkey[h], kEmpty, key);
        if (prev == kEmpty || prev == key) return (int)h;
      }
      h = (h + 1) & (kDH - 1);
    }
    return -1;
  };
  bool bad = false;
  // 4 entries per thread per round: every locate, then every key load in flight, then the
  // probes (one memory round trip per round instead of one per entry)
  constexpr int kLB = 4;
  for (uint32_t c0 = 0; c0 < E; c0 += kBkThr * kLB) {
    int32_t id[kLB];
    uint32_t kk[kLB];
#pragma unroll
    for (int q = 0; q < kLB; ++q) {
      const uint32_t g = c0 + q * kBkThr + t;
      id[q] = locate(g < E ? g : E - 1);
    }
#pragma unroll
    for (int q = 0; q < kLB; ++q) kk[q] = tkeys[id[q]];
#pragma unroll
    for (int q = 0; q < kLB; ++q)
      if (c0 + q * kBkThr + t < E) bad |= probe(kk[q] | (hb << shift), true) < 0;
  }
  __syncthreads();
  // key index j of every occupied slot (strided: conflict-free LDS reads): compaction
  // order, or (sorted) the key's rank = # smaller keys of the unit (the keys are
  // distinct and below kEmpty)
  constexpr int kPer = kDH / kBkThr;
  uint32_t cc = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q) cc += hkey[q * kBkThr + t] != kEmpty;
  uint32_t D;
  uint32_t wd = tp_block_scan<kBkThr>(cc, lds, &D);
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int s = q * kBkThr + t;
    const uint32_t k = hkey[s];
    if (k != kEmpty) {
      uint32_t j = wd++;
      if (sorted) {
        j = 0;
        for (int r = 0; r < kDH; ++r) j += hkey[r] < k;  // (kEmpty is never < k)
      }
      hmap[s] = j;
      uo[j] = key0 | k;
    }
  }
  __syncthreads();
  const uint32_t room = eoff < (uint32_t)tpf::kEC ? tpf::kEC - eoff : 0u;
  bad |= E > room;
  const uint32_t Er = E < room ? E : room;
  for (uint32_t c0 = 0; c0 < Er; c0 += kBkThr * kLB) {
    int32_t id[kLB];
    uint32_t kk[kLB];
#pragma unroll
    for (int q = 0; q < kLB; ++q) {
      const uint32_t g = c0 + q * kBkThr + t;
      id[q] = locate(g < Er ? g : Er - 1);
    }
#pragma unroll
    for (int q = 0; q < kLB; ++q) kk[q] = tkeys[id[q]];
#pragma unroll
    for (int q = 0; q < kLB; ++q) {
      const uint32_t g = c0 + q * kBkThr + t;
      if (g >= Er) continue;
      const int h = probe(kk[q] | (hb << shift), false);
      po[eoff + g] = id[q];
      jo[eoff + g] = h >= 0 ? (uint16_t)hmap[h] : (uint16_t)0;
    }
  }
  if (bad) atomicOr(err, 1);
  if (t == 0) {
    co[0] = (int32_t)D;
    co[1] = (int32_t)(E < room ? E : room);
  }
  __syncthreads();
  return E < room ? E : room;
}

// Rank order of a unit's distinct keys by counting them into 256 bins of their top bits
// (the mixed keys are uniform over the unit's range [0, 2^kbits)) and comparing each key
// with the few others of its bin: O(D) work and 5 barriers instead of tp_bk_ranksort's
// O(D^2) scan. In: dl[0..D) (key u32 << 32 | count | slot). Out: dl[0..D) in key order.
// Scratch: sc = the dead hash region (>= kDH + 514 words: bin keys, counts, starts).
__device__ __forceinline__ void tpf_rank_binned(uint64_t* dl, uint32_t* sc, uint32_t D, int kbits,
                                                uint32_t* lds) {
  using namespace tp;
  constexpr int kPerT = kDH / kBkThr;  // <= 4 keys per thread
  const int t = threadIdx.x;
  const int bsh = kbits > 8 ? kbits - 8 : 0;
  uint32_t* bkey = sc;              // [kDH] keys grouped by bin
  uint32_t* bcnt = sc + kDH;        // [256]
  uint32_t* bst = bcnt + 256;       // [256] bin starts
  if (t < 256) bcnt[t] = 0u;
  __syncthreads();
  uint64_t e[kPerT];
  uint32_t bs[kPerT];  // bin << 16 | slot in bin
#pragma unroll
  for (int q = 0; q < kPerT; ++q) {
    const uint32_t i = q * kBkThr + t;
    e[q] = i < D ? dl[i] : 0ull;
    if (i < D) {
      const uint32_t bin = ((uint32_t)(e[q] >> 32) >> bsh) & 255u;
      bs[q] = bin << 16 | atomicAdd(&bcnt[bin], 1u);
    }
  }
  __syncthreads();
  uint32_t tot;
  const uint32_t st = tp_block_scan<kBkThr>(t < 256 ? bcnt[t] : 0u, lds, &tot);
  if (t < 256) bst[t] = st;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kPerT; ++q)
    if (q * kBkThr + t < D) bkey[bst[bs[q] >> 16] + (bs[q] & 0xffffu)] = (uint32_t)(e[q] >> 32);
  __syncthreads();
  uint32_t rk[kPerT];
#pragma unroll
  for (int q = 0; q < kPerT; ++q) {
    if (q * kBkThr + t >= D) continue;
    const uint32_t bin = bs[q] >> 16, a = bst[bin], n = bcnt[bin];
    const uint32_t k = (uint32_t)(e[q] >> 32);
    uint32_t r = a;
    for (uint32_t m = 0; m < n; ++m) r += bkey[a + m] < k;  // distinct keys
    rk[q] = r;
  }
  __syncthreads();  // (every dl entry is in registers: dl takes the ordered list)
#pragma unroll
  for (int q = 0; q < kPerT; ++q)
    if (q * kBkThr + t < D) dl[rk[q]] = e[q];
  __syncthreads();
}

// a unit key's bits (the bucket build's units carry the key's occurrences in the top byte
// until the tail filter rewrites them)
constexpr uint64_t kUoKey = (1ull << 56) - 1;

// The unit's sketch traffic with global atomics (units of more than kFlD keys, or k != 2):
// insert and query with the keys strided over the threads (key j = q * kBkThr + t), two
// keys at a time (4 spill past 64 VGPRs); keep flags -> occ[].
__device__ __forceinline__ void tpf_filter_global(const uint64_t* __restrict__ uo, uint32_t D,
                                                  const CmArgs& cm, uint32_t* occ) {
  using namespace tp;
  constexpr int kKP = tpf::kUnitK / kBkThr;
  const int t = threadIdx.x;
  auto load2 = [&](int hq, uint64_t (&k2)[2], uint32_t (&c2)[2]) -> uint32_t {
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t j = (hq + i) * kBkThr + t;
      k2[i] = j < D ? uo[j] & kUoKey : 0ull;
      c2[i] = j < D ? (occ[j] > 255u ? 255u : occ[j]) : 0u;
      v |= (j < D ? 1u : 0u) << i;
    }
    return v;
  };
#pragma unroll
  for (int hq = 0; hq < kKP; hq += 2) {
    uint64_t k2[2];
    uint32_t c2[2];
    const uint32_t v = load2(hq, k2, c2);
    if (!v) continue;
    if (cm.k == kCmBatchK && cm.ncells32) {
      cm_insert_batch<2>(cm, k2, c2, v);
    } else {
      for (int i = 0; i < 2; ++i)
        if ((v >> i) & 1u) cm_insert_key(cm, k2[i], c2[i]);
    }
  }
  __syncthreads();  // every insert of this minibatch that can reach these keys' cells is done
#pragma unroll
  for (int hq = 0; hq < kKP; hq += 2) {
    uint64_t k2[2];
    uint32_t c2[2], e2[2] = {0u, 0u};
    const uint32_t v = load2(hq, k2, c2);
    if (!v) continue;
    if (cm.k == kCmBatchK && cm.ncells32) {
      cm_query_batch<2>(cm, k2, v, e2);
    } else {
      for (int i = 0; i < 2; ++i) e2[i] = (v >> i) & 1u ? cm_query_key(cm, k2[i]) : 0u;
    }
    // (each thread reads back only its own occ words: no barrier between the two)
    for (int i = 0; i < 2; ++i)
      if ((v >> i) & 1u) occ[(hq + i) * kBkThr + t] = (int)e2[i] > cm.freq ? 1u : 0u;
  }
}

// The unit's sketch traffic staged in LDS (units of <= kFlD keys, k = 2): the distinct
// sketch words of the unit's cells go into an LDS table (word index -> value), each
// loaded ONCE from HBM by the thread that claimed its slot; the saturating adds are LDS
// CAS loops, the queries read the table, and the changed words are written back with
// plain stores. Valid because this workgroup owns every region its keys map to
// (countmin.cuh) and no other kernel touches the sketch meanwhile (the tail-filtered
// pipelines order their bucket kernels): one memory round trip per key instead of the
// global form's load -> CAS -> reload chain (a device-scope atomic drops the line from the
// XCD's L2, MI355X_MICROARCH.md: the reload crosses the fabric again).
constexpr int kFlD = 1024;    // keys of a staged unit (occ_small: the dead entry-hash LDS)
constexpr int kFlTab = 4096;  // word table slots (load <= 0.5)

__device__ __forceinline__ void lds_sat_add_byte(uint32_t* w, uint32_t sh, uint32_t cnt,
                                                 uint32_t vmax) {
  uint32_t old = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (true) {
    const uint32_t b = (old >> sh) & 0xffu;
    const uint32_t nb = (cnt > vmax - b) ? vmax : b + cnt;
    if (nb == b) return;
    const uint32_t prev = atomicCAS(w, old, (old & ~(0xffu << sh)) | (nb << sh));
    if (prev == old) return;
    old = prev;
  }
}

// (the staged form in two halves: claim + gathers in flight, issued before the unit's
// occurrence counting so the two memory round trips overlap; then adds, query, write-back)
struct CmStage {
  static constexpr int kQ = kFlD / tp::kBkThr;  // keys per thread (strided)
  uint32_t cell[kQ][kCmBatchK], g[kQ][kCmBatchK];
  uint32_t sl[kQ];         // the two probes' table slots, 16 bits each
  uint32_t mine, valid;    // (packed: registers are live across the occurrence counting)
  __device__ __forceinline__ uint32_t slot(int q, int p) const {
    return (sl[q] >> (16 * p)) & 0xffffu;
  }
};

__device__ __forceinline__ void cm_stage_begin(const uint64_t* __restrict__ uo, uint32_t D,
                                               const CmArgs& cm, uint32_t* wkey, CmStage& st,
                                               uint32_t* occ_packed) {
  using namespace tp;
  constexpr int kQ = CmStage::kQ;
  const int t = threadIdx.x;
  uint64_t k[kQ];
  st.valid = 0;
  st.mine = 0;
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    const uint32_t j = q * kBkThr + t;
    const uint64_t raw = uo[j < D ? j : 0];  // (D >= 1 here; clamped, unconditional loads)
    k[q] = raw & kUoKey;
    // (packed unit: the key's occurrence count rides in the top byte -- no second pass)
    if (occ_packed && j < D) occ_packed[j] = (uint32_t)(raw >> 56);
    st.valid |= (j < D ? 1u : 0u) << q;
  }
  cm_cells_batch<kQ>(cm, k, st.cell);
#pragma unroll
  for (int q = 0; q < kQ; ++q)
#pragma unroll
    for (int p = 0; p < kCmBatchK; ++p) {
      if (p == 0) st.sl[q] = 0;
      if (!((st.valid >> q) & 1u)) continue;
      const uint32_t w1 = (st.cell[q][p] >> 2) + 1u;  // (< 2^30 words: ncells32)
      uint32_t h = (w1 * 0x9E3779B1u) >> (32 - 12);
      static_assert(kFlTab == 1 << 12, "table hash width");
      while (true) {
        const uint32_t prev = atomicCAS(&wkey[h], 0u, w1);
        if (prev == 0u) {
          st.mine |= 1u << (q * kCmBatchK + p);
          break;
        }
        if (prev == w1) break;
        h = (h + 1) & (kFlTab - 1);
      }
      st.sl[q] |= h << (16 * p);
    }
#pragma unroll
  for (int q = 0; q < kQ; ++q)
#pragma unroll
    for (int p = 0; p < kCmBatchK; ++p)  // (every claimed word's load in flight)
      st.g[q][p] = (st.mine >> (q * kCmBatchK + p)) & 1u
                       ? __hip_atomic_load(cm.cells + (st.cell[q][p] >> 2), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT)
                       : 0u;
}

__device__ __forceinline__ void cm_stage_end(const CmArgs& cm, uint32_t* occ, uint32_t* wval,
                                             CmStage& st) {
  using namespace tp;
  constexpr int kQ = CmStage::kQ;
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < kQ; ++q)
#pragma unroll
    for (int p = 0; p < kCmBatchK; ++p)
      if ((st.mine >> (q * kCmBatchK + p)) & 1u) wval[st.slot(q, p)] = st.g[q][p];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    if (!((st.valid >> q) & 1u)) continue;
    const uint32_t o = occ[q * kBkThr + t];
    const uint32_t c = o > 255u ? 255u : o;
#pragma unroll
    for (int p = 0; p < kCmBatchK; ++p)
      lds_sat_add_byte(&wval[st.slot(q, p)], (st.cell[q][p] & 3u) * 8u, c, cm.vmax);
  }
  __syncthreads();  // every insert of the unit is in the table
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    if (!((st.valid >> q) & 1u)) continue;
    uint32_t r = cm.vmax;
#pragma unroll
    for (int p = 0; p < kCmBatchK; ++p) {
      const uint32_t v = (wval[st.slot(q, p)] >> ((st.cell[q][p] & 3u) * 8u)) & 0xffu;
      r = v < r ? v : r;
    }
    occ[q * kBkThr + t] = (int)r > cm.freq ? 1u : 0u;  // (own occ words: read above)
  }
#pragma unroll
  for (int q = 0; q < kQ; ++q)
#pragma unroll
    for (int p = 0; p < kCmBatchK; ++p)
      if ((st.mine >> (q * kCmBatchK + p)) & 1u) {
        const uint32_t v = wval[st.slot(q, p)];
        if (v != st.g[q][p]) cm.cells[st.cell[q][p] >> 2] = v;
      }
}

// Fused tail-feature filter of one unit of the flat layout (reference
// MinibatchReader::read, src/learner/sgd.h:131-150: CountMin insertKeys of the minibatch's
// per-key counts, then queryKeys > tail_feature_freq, src/parameter/frequency_filter.h:
// 26-45). In: keys uo[0..D), entries po / jo[ein .. ein + E) (jo = key index), the tile
// kernel's per-entry occurrence counts ecnt. Each key's count (its entries' counts,
// saturated to a byte) goes into the partitioned sketch (countmin.cuh: this workgroup owns
// every region its keys map to), then after a barrier every key is queried. Out: the kept
// keys at uo[0..D') in their order (sorted stays sorted), the kept entries at
// po / jo[eout .. eout + E') with the new key indices, and w_ent = 0 at the filtered
// entries -- the minibatch as if the filtered keys were absent, so the step, pack and
// owner kernels need no change. (D', E') -> res[0..1] (LDS).
__device__ __forceinline__ void tpf_filter_unit(uint64_t* __restrict__ uo, int32_t* __restrict__ po,
                                                uint16_t* __restrict__ jo, uint32_t D, uint32_t E,
                                                uint32_t ein, uint32_t eout,
                                                const uint8_t* __restrict__ ecnt, const CmArgs& cm,
                                                float* __restrict__ w_ent, int64_t w_cap,
                                                uint32_t* occ_big, uint32_t* occ_small,
                                                uint32_t* wkey, uint32_t* wval, uint32_t* lds,
                                                uint32_t* res, bool packed) {
  using namespace tp;
  constexpr int kKP = tpf::kUnitK / kBkThr;  // 4 keys per thread (contiguous)
  constexpr int kEP = 4;                      // entries per thread per chunk
  constexpr uint32_t kNone = 0xffffffffu;
  const int t = threadIdx.x;
  // the sketch words of the unit staged in LDS (block-uniform choice): <= kFlD keys
  const bool staged = D <= (uint32_t)kFlD && cm.k == kCmBatchK && cm.ncells32;
  uint32_t* occ = staged ? occ_small : occ_big;
  if (staged)
    for (uint32_t s = t; s < (uint32_t)kFlTab; s += kBkThr) wkey[s] = 0u;
  if (!packed)
    for (uint32_t j = t; j < D; j += kBkThr) occ[j] = 0u;
  __syncthreads();
  CmStage st;
  const bool stage = staged && D > 0;
  if (stage) cm_stage_begin(uo, D, cm, wkey, st, packed ? occ : nullptr);
  // occurrences per key: from the keys' top byte (packed: the LDS build summed them), or
  // 4 entries per thread per round, every load of a round in flight (clamped addresses,
  // selects afterwards)
  if (packed && !stage) {
    for (uint32_t j = t; j < D; j += kBkThr) occ[j] = (uint32_t)(uo[j] >> 56);
  }
  for (uint32_t c0 = 0; c0 < (packed ? 0u : E); c0 += kBkThr * 4) {
    uint32_t gi[4], jj[4], ec[4];
    int32_t id[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t g = c0 + q * kBkThr + t;
      gi[q] = ein + (g < E ? g : E - 1);
      id[q] = po[gi[q]];
      jj[q] = jo[gi[q]];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) ec[q] = ecnt[id[q]];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (c0 + q * kBkThr + t < E) atomicAdd(&occ[jj[q]], ec[q]);
  }
  __syncthreads();
  if (stage) {
    cm_stage_end(cm, occ, wval, st);
  } else if (D > 0 && !staged) {
    tpf_filter_global(uo, D, cm, occ);
  }
  __syncthreads();
  uint64_t key[kKP];
  uint32_t keep = 0, kc = 0;
#pragma unroll
  for (int q = 0; q < kKP; ++q) {  // contiguous keys per thread for the compaction
    const uint32_t j = t * kKP + q;
    key[q] = j < D ? uo[j] & kUoKey : 0ull;
    if (j < D && occ[j]) {
      keep |= 1u << q;
      ++kc;
    }
  }
  uint32_t Dn;
  uint32_t off = tp_block_scan<kBkThr>(kc, lds, &Dn);  // (barriers: every uo read is done)
#pragma unroll
  for (int q = 0; q < kKP; ++q) {
    const uint32_t j = t * kKP + q;
    if (j < D) {
      const bool k = (keep >> q) & 1u;
      occ[j] = k ? off : kNone;
      if (k) uo[off++] = key[q];
    }
  }
  __syncthreads();
  uint32_t eo = 0;
  for (uint32_t c0 = 0; c0 < E; c0 += kBkThr * kEP) {
    int32_t id[kEP];
    uint32_t nj[kEP], ec = 0;
#pragma unroll
    for (int q = 0; q < kEP; ++q) {
      const uint32_t g = c0 + t * kEP + q;
      nj[q] = kNone;
      id[q] = 0;
      if (g < E) {
        id[q] = po[ein + g];
        nj[q] = occ[jo[ein + g]];
        if (nj[q] != kNone) ++ec;
        else if (in_range(id[q], w_cap)) w_ent[id[q]] = 0.f;
      }
    }
    uint32_t tot;
    uint32_t o = eout + eo + tp_block_scan<kBkThr>(ec, lds, &tot);  // (reads done: barrier)
#pragma unroll
    for (int q = 0; q < kEP; ++q)
      if (nj[q] != kNone) {  // (output positions <= input ones: compaction)
        po[o] = id[q];
        jo[o] = (uint16_t)nj[q];
        ++o;
      }
    eo += tot;
  }
  if (t == 0) {
    res[0] = Dn;
    res[1] = eo;
  }
  __syncthreads();
}

// One workgroup per pair of fine buckets (pair = 0: per fine bucket), the tp_bucket
// geometry and build; the occupied hash slots in compaction order are the keys' indices.
// kFilt (tail filter, count mode): the LDS build sums the tile kernel's per-entry
// occurrence counts, and each key of a built unit carries its count (a byte) in the top
// byte of uniqf for tpf_filter_kernel, which runs as its own launch so that only IT has to
// run in minibatch order.
template <bool kFilt>
__global__ void __launch_bounds__(tp::kBkThr, 8)
tpf_bucket_kernel(const uint32_t* __restrict__ tkeys, const uint16_t* __restrict__ toff, int nbf,
                  int pair, int T, int shift, uint64_t* __restrict__ uniqf,
                  int32_t* __restrict__ ent_pos, uint16_t* __restrict__ ent_j,
                  int32_t* __restrict__ cnt, int32_t* __restrict__ err, int sorted,
                  const uint8_t* __restrict__ ecnt) {
  using namespace tp;
  __shared__ alignas(16) uint16_t eh[kECapL];  // hash slot of every gathered entry
  __shared__ uint64_t hs[kDH];     // hash (key u32 | count u32 -> key index)
  __shared__ uint64_t dl[kDH];     // per-tile runs, then the compacted occupied slots
  __shared__ uint32_t lds[kBkThr / 64 + 1];
  __shared__ uint32_t flag;
  uint32_t* hkey = reinterpret_cast<uint32_t*>(hs);
  uint32_t* hcnt = hkey + kDH;
  const int t = threadIdx.x, b = blockIdx.x;
  const int f0 = pair ? 2 * b : b;
  const uint64_t key0 = (uint64_t)f0 << shift;
  uint64_t* uo = uniqf + (int64_t)b * tpf::kUC;
  int32_t* po = ent_pos + (int64_t)b * tpf::kEC;
  uint16_t* jo = ent_j + (int64_t)b * tpf::kEC;
  int32_t* co = cnt + (int64_t)b * 4;
  int32_t idx[kG];
  uint32_t E, D;
  const bool good = tp_bk_build<kFilt>(tkeys, toff, nbf, T, shift, f0, pair ? 2 : 1, 0u, hkey,
                                       hcnt, dl, eh, lds, &flag, idx, &E, &D, nullptr, ecnt);
  if (good) {
    // key index j: compaction order, or (sorted: the multi-GPU exchange rows must be
    // key-ordered) the rank order of tp_bk_ranksort; slot -> j in LDS (the dead hash
    // counts, or the dead compaction list once it is sorted into hs)
    uint32_t* jmap = hcnt;
    const uint64_t* lst = dl;
    if (sorted && D > 64) {  // binned rank order into dl; the dead hash takes slot -> j
      tpf_rank_binned(dl, hkey, D, pair ? shift + 1 : shift, lds);
      jmap = hkey;
    } else if (sorted) {
      tp_bk_ranksort(dl, hs, D);
      __syncthreads();
      jmap = reinterpret_cast<uint32_t*>(dl);
      lst = hs;
    }
    for (uint32_t j = t; j < D; j += kBkThr) {
      const uint64_t v = lst[j];
      // (tail filter: the key's occurrences, saturated to a byte, ride in the top byte
      // until the filter rewrites the unit's keys)
      uo[j] = key0 | (uint32_t)(v >> 32) |
              (kFilt ? (uint64_t)min((uint32_t)(v >> 16) & 0xffffu, 255u) << 56 : 0ull);
      jmap[(uint32_t)v & 0xffffu] = j;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kG; ++q) {
      if (idx[q] < 0) continue;
      const uint32_t g = q * kBkThr + t;
      po[g] = idx[q];
      jo[g] = (uint16_t)jmap[eh[g]];
    }
    if (t == 0) {
      co[0] = (int32_t)D;
      co[1] = (int32_t)E;
      co[2] = 0;
      co[3] = 0;
    }
  } else {
    // the pair's entries overflow the LDS capacity or its hash (near-distinct keys; the
    // hash build gives up after kBkProbe probes): its fine buckets one after the other,
    // each a unit with its own key index space. (Measured and not kept: the LDS build per
    // fine bucket here -- as a second inlined build it spilled the main path, as a
    // non-inlined call (308 B of scratch) it slowed the headline step 0.082 -> 0.105 ms,
    // profiles/r6_skew_layout.log.)
    {
      const uint32_t e0 = tpf_unit_light(tkeys, toff, nbf, T, shift, f0, 0u, key0, hkey, hcnt, eh,
                                         lds, uo, po, jo, 0u, co, err, sorted != 0);
      if (pair)
        tpf_unit_light(tkeys, toff, nbf, T, shift, f0 + 1, 1u, key0, hkey, hcnt, eh, lds,
                       uo + tpf::kUnitK, po, jo, e0, co + 2, err, sorted != 0);
      else if (t == 0) {
        co[2] = 0;
        co[3] = 0;
      }
    }
  }
}

// The fused tail filter of every bucket workgroup's units (tpf_filter_unit), one
// workgroup per bucket group, after tpf_bucket_kernel<true>: the partitioned CountMin
// insert + query of the minibatch's keys and the compaction of the filtered ones. A launch
// of its own so that only the sketch traffic runs in minibatch order (the callers chain
// these launches across their preparation streams; the bucket builds overlap freely):
// ordering the whole bucket kernel cost the pipelined step ~6.5 us
// (profiles/r6_tail_filter.log). cnt_pre <- the unfiltered counts, cnt <- the kept ones.
__global__ void __launch_bounds__(tp::kBkThr, 8)
tpf_filter_kernel(uint64_t* __restrict__ uniqf, int32_t* __restrict__ ent_pos,
                  uint16_t* __restrict__ ent_j, int32_t* __restrict__ cnt,
                  const uint8_t* __restrict__ ecnt, CmArgs cm, float* __restrict__ w_ent,
                  int64_t w_cap, int32_t* __restrict__ cnt_pre) {
  using namespace tp;
  __shared__ uint64_t hs[kDH];          // occ_big / the sketch table's values
  __shared__ uint64_t dl[kDH];          // the sketch table's word ids
  __shared__ uint32_t occs[kFlD];       // occ_small
  __shared__ uint32_t lds[kBkThr / 64 + 3];
  static_assert(kFlTab * 4 <= kDH * 8, "filter LDS");
  const int t = threadIdx.x, b = blockIdx.x;
  uint64_t* uo = uniqf + (int64_t)b * tpf::kUC;
  int32_t* po = ent_pos + (int64_t)b * tpf::kEC;
  uint16_t* jo = ent_j + (int64_t)b * tpf::kEC;
  int32_t* co = cnt + (int64_t)b * 4;
  const uint32_t D0 = (uint32_t)co[0], E0 = (uint32_t)co[1];
  const uint32_t D1 = (uint32_t)co[2], E1 = (uint32_t)co[3];
  // a unit the LDS build wrote carries its keys' counts in the top byte (every count >= 1);
  // the register-light units do not (their counts come from the entries)
  const bool packed = D0 > 0 && (uo[0] >> 56) != 0;
  uint32_t* occ = reinterpret_cast<uint32_t*>(hs);
  uint32_t* wkey = reinterpret_cast<uint32_t*>(dl);
  uint32_t* res = lds + kBkThr / 64 + 1;
  tpf_filter_unit(uo, po, jo, D0, E0, 0u, 0u, ecnt, cm, w_ent, w_cap, occ, occs, wkey, occ, lds,
                  res, packed);
  const uint32_t D0k = res[0], E0k = res[1];
  uint32_t D1k = 0, E1k = 0;
  if (D1 | E1) {
    __syncthreads();
    tpf_filter_unit(uo + tpf::kUnitK, po, jo, D1, E1, E0, E0k, ecnt, cm, w_ent, w_cap, occ, occs,
                    wkey, occ, lds, res, false);
    D1k = res[0];
    E1k = res[1];
  }
  if (t == 0) {
    if (cnt_pre) {  // the unfiltered counts (the exchange rows are sized from them)
      int32_t* cp = cnt_pre + (int64_t)b * 4;
      cp[0] = (int32_t)D0;
      cp[1] = (int32_t)E0;
      cp[2] = (int32_t)D1;
      cp[3] = (int32_t)E1;
    }
    co[0] = (int32_t)D0k;
    co[1] = (int32_t)E0k;
    co[2] = (int32_t)D1k;
    co[3] = (int32_t)E1k;
  }
}

// Lookup-or-insert of one key with ONE 16-B load per probe (key and weight of the slot
// together; resolve_key reads the weight after the key compare, a second round trip).
__device__ __forceinline__ uint32_t tpf_resolve(Slot* __restrict__ slots, uint64_t mask,
                                                uint64_t home_base, uint64_t home_m, int home_shr,
                                                uint64_t h, int init_type, float init_v,
                                                float init_s, uint64_t seed, float* w, int* ins) {
  uint64_t idx = home_slot(h, mask, home_base, home_m, home_shr) & mask;
  *w = 0.f;
  for (uint64_t probe = 0; probe <= mask; ++probe) {
    const uint4 v = *reinterpret_cast<const uint4*>(&slots[idx]);
    const uint64_t k = ((uint64_t)v.y << 32) | v.x;
    if (k == h) {  // (non-zero init: the weight once its inserter published it)
      *w = init_type == kInitZero ? __uint_as_float(v.z)
                                  : published_w(&slots[idx], h, init_type, init_v, init_s, seed);
      return (uint32_t)idx;
    }
    if (k == kEmptyKey) {
      const unsigned long long prev = atomicCAS((unsigned long long*)&slots[idx].key,
                                                (unsigned long long)kEmptyKey,
                                                (unsigned long long)h);
      if (prev == kEmptyKey) {
        if (init_type != kInitZero) {
          *w = init_value(h, init_type, init_v, init_s, seed);
          publish_init(&slots[idx], *w);
        }
        ++*ins;
        return (uint32_t)idx;
      }
      if (prev == h) {  // claimed by another lane meanwhile
        *w = published_w(&slots[idx], h, init_type, init_v, init_s, seed);
        return (uint32_t)idx;
      }
    }
    idx = (idx + 1) & mask;
  }
  return tpf::kNoSlot;
}

// The step boundary of the flat 1-GPU path, one 256-thread workgroup per bucket
// workgroup region (replaces tp_seg_update + kv_resolve: one launch, no global atomics):
//   update A   every unit: the entries' partials psum[ent_pos] go into per-key LDS
//              accumulators in 64-bit fixed point (scale 2^(48 - e) from the unit's
//              largest |partial| < 2^e: <= 8192 addends stay below 2^61; exact,
//              order-independent sums), then the optimizer update of each key at the
//              slot its pull resolved (slotA), with the update statistics
//   pull B     every unit: lookup-or-insert of B's keys -> slotB, weights into LDS, then
//              scattered to B's tile-entry order: w_ent[ent_pos] = w[ent_j]
// A and B must share the bucket geometry (same minibatch size); either half may be off
// (the first pull, the last update). Block 0 also turns A's AUC histogram into metrics.
// Within a workgroup the update's slot stores are visible to the pull's loads after the
// barrier (workgroup scope: same CU, write-through L1).
__global__ void __launch_bounds__(tpf::kThr)
tpf_step_kernel(int do_upd, const int32_t* __restrict__ cntA, const int32_t* __restrict__ posA,
                const uint16_t* __restrict__ jA, const uint32_t* __restrict__ slotA,
                const float* __restrict__ psum, int64_t p_cap, int do_res,
                const int32_t* __restrict__ cntB, const uint64_t* __restrict__ uniqB,
                const int32_t* __restrict__ posB, const uint16_t* __restrict__ jB,
                uint32_t* __restrict__ slotB, float* __restrict__ w_ent, int64_t w_cap,
                Slot* __restrict__ slots, uint64_t mask, uint64_t home_base, uint64_t home_m,
                int home_shr, int init_type, float init_v, float init_s, uint64_t seed,
                int32_t* __restrict__ err, int32_t* __restrict__ inserted, UpdateParams p,
                double* __restrict__ stats, int acc_stripes, uint32_t* __restrict__ hist,
                int nbins, int hist_stripes, double* __restrict__ metrics,
                int64_t* __restrict__ step_counter) {
  using namespace tpf;
  __shared__ long long acc[kUnitK];  // fixed-point gradient sums of a unit's keys
  __shared__ float wj[kUnitK];       // pulled weights of a unit's keys
  __shared__ uint32_t smax;
  const int t = threadIdx.x, b = blockIdx.x, lane = t & 63;
  // the step's AUC epilogue in an extra last workgroup of its own (tpf_step launches
  // groups + 1): in unit 0's workgroup its 8 dependent stripe loads delayed that unit
  if (do_upd && hist && b == (int)gridDim.x - 1) {
    auc_hist_block(hist, nbins, hist_stripes, metrics, step_counter);
    return;
  }
  double dnnz = 0, wsum = 0, dsum = 0;
  if (do_upd) {
    const int32_t* c = cntA + (int64_t)b * 4;
#pragma unroll 1
    for (int s = 0; s < 2; ++s) {
      // (counts clamped to the regions: a corrupted count never leaves them)
      const int e0 = s ? min(max(c[1], 0), kEC) : 0;
      const int D = min(c[2 * s], kUnitK), E = min(c[2 * s + 1], kEC - e0);
      if (D <= 0) continue;
      const int64_t eb = (int64_t)b * kEC + e0;
      const int64_t kb = (int64_t)b * kUC + s * kUnitK;
      for (int j = t; j < D; j += kThr) acc[j] = 0ll;
      if (t == 0) smax = 0u;
      constexpr int kR = 8;  // entries held in registers per thread (<= 2048 per unit)
      float v[kR];
      uint16_t jj[kR];
      int32_t pos[kR];
      float vmax = 0.f;
      // two batches of unconditional loads at clamped in-region addresses (a guarded
      // load per entry compiled to a branch + s_waitcnt each: 2 x kR serialised round
      // trips), then selects
      const int64_t rb = (int64_t)b * kEC;  // (always inside the entry region)
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        const int g = r * kThr + t;
        const int64_t gi = g < E ? eb + g : rb;
        pos[r] = posA[gi];
        jj[r] = jA[gi];
      }
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        const bool ok = r * kThr + t < E && in_range(pos[r], p_cap);
        const float x = psum[ok ? pos[r] : 0];
        v[r] = ok ? x : 0.f;
        if (r * kThr + t >= E) jj[r] = 0;
      }
#pragma unroll
      for (int r = 0; r < kR; ++r) vmax = fmaxf(vmax, fabsf(v[r]));
      for (int g = kR * kThr + t; g < E; g += kThr) {
        const int32_t pos = posA[eb + g];
        if (in_range(pos, p_cap)) vmax = fmaxf(vmax, fabsf(psum[pos]));
      }
      __syncthreads();  // acc / smax zeroed
      fx_tile_max(vmax, &smax);
      __syncthreads();
      const int k2 = fx_shift(smax);
      const double sc = ldexp(1.0, k2);
#pragma unroll
      for (int r = 0; r < kR; ++r)
        if (v[r] != 0.f && jj[r] < kUnitK) fx_add(acc, jj[r], v[r], sc);
      for (int g = kR * kThr + t; g < E; g += kThr) {
        const int32_t pos = posA[eb + g];
        const uint16_t j = jA[eb + g];
        const float x = in_range(pos, p_cap) ? psum[pos] : 0.f;
        if (x != 0.f && j < kUnitK) fx_add(acc, j, x, sc);
      }
      __syncthreads();
      const double isc = ldexp(1.0, -k2);
      for (int j = t; j < D; j += kThr) {
        const uint32_t si = slotA[kb + j];
        if (si == kNoSlot || si > mask) continue;
        const float gs = (float)((double)acc[j] * isc) * p.grad_scale;
        if (gs != gs) continue;
        Slot sl = slots[si];
        const float w_old = apply_update(sl, gs, p);
        slots[si] = sl;
        dnnz += (double)((sl.w != 0.f) - (w_old != 0.f));
        wsum += (double)sl.w * sl.w;
        const double d = (double)sl.w - w_old;
        dsum += d * d;
      }
      __syncthreads();  // (acc of the next unit; the pull reads these slots)
    }
  }
  int ins = 0;
  if (do_res) {
    const int32_t* c = cntB + (int64_t)b * 4;
#pragma unroll 1
    for (int s = 0; s < 2; ++s) {
      const int e0 = s ? min(max(c[1], 0), kEC) : 0;
      const int D = min(c[2 * s], kUnitK), E = min(c[2 * s + 1], kEC - e0);
      if (D <= 0) continue;
      const int64_t eb = (int64_t)b * kEC + e0;
      const int64_t kb = (int64_t)b * kUC + s * kUnitK;
      for (int j = t; j < D; j += kThr) {
        float w;
        const uint32_t si = tpf_resolve(slots, mask, home_base, home_m, home_shr, uniqB[kb + j],
                                        init_type, init_v, init_s, seed, &w, &ins);
        if (si == kNoSlot && err) atomicOr(err, 1);  // table full
        slotB[kb + j] = si;
        wj[j] = w;
      }
      __syncthreads();
      const int64_t rb = (int64_t)b * kEC;
      for (int g0 = 0; g0 < E; g0 += 8 * kThr) {  // (8 entries per thread: loads batched)
        int32_t pp[8];
        uint16_t jq[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int g = g0 + q * kThr + t;
          const int64_t gi = g < E ? eb + g : rb;
          pp[q] = posB[gi];
          jq[q] = jB[gi];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (g0 + q * kThr + t < E && in_range(pp[q], w_cap) && jq[q] < kUnitK)
            w_ent[pp[q]] = wj[jq[q]];
      }
      __syncthreads();  // (wj of the next unit)
    }
  }
  if (do_upd && stats) {
    const double a = wave_sum_dpp(dnnz), bb = wave_sum_dpp(wsum), cc = wave_sum_dpp(dsum);
    if (lane == 63) {
      double* st = acc_stripe(stats, acc_stripes);
      if (a != 0) atomicAdd(&st[0], a);
      if (bb != 0) atomicAdd(&st[1], bb);
      if (cc != 0) atomicAdd(&st[2], cc);
    }
  }
  if (inserted) {
    const int tot = wave_sum(ins);
    if (lane == 0 && tot) atomicAdd(inserted, tot);
  }
}

// Overlapped form of tpf_step_kernel (opt-in, PSAMD_TPF_STEP2=1: measured SLOWER, see
// tpf_step below; the chain-latency model that motivated it did not hold): the dependent global-load chains of
// the step run together instead of one after another. tpf_step_kernel walks unit 0's
// update, unit 1's update, unit 0's pull, unit 1's pull, each a chain of dependent
// loads (entry -> partial; key -> slot record; key -> hash probe) behind barriers: ~12
// load latencies per workgroup, with ~114 keys and ~500 entries per unit too little
// work to hide them (19 us per half, profiles/r4_flat_ab.log). Here both units are one
// flat index space and, before the first barrier, every thread issues its A entries'
// partial loads, its A keys' slot records and its B keys' hash probes (lookup-or-insert:
// the slot a key resolves to does not depend on A's update), so the chain is about
// four latencies: prefetch | LDS fixed-point sums | update + store | re-read of the
// weights of B keys that existed (A may have updated them) | scatter. The pulled
// weights reuse the accumulators' LDS. Same results as tpf_step_kernel (same
// per-unit scales, same fixed-point sums, same per-key update).
namespace tpf2 {
constexpr int kRE = 8;   // A entries held in registers per thread (2048 per workgroup)
constexpr int kRS = 2;   // A slot records held in registers per thread (512 keys)
constexpr int kRP = 4;   // B probes held in registers per thread (1024 keys)
constexpr int kRB = 8;   // B entries held in registers per thread
}  // namespace tpf2

__global__ void __launch_bounds__(tpf::kThr)
tpf_step2_kernel(int do_upd, const int32_t* __restrict__ cntA, const int32_t* __restrict__ posA,
                 const uint16_t* __restrict__ jA, const uint32_t* __restrict__ slotA,
                 const float* __restrict__ psum, int64_t p_cap, int do_res,
                 const int32_t* __restrict__ cntB, const uint64_t* __restrict__ uniqB,
                 const int32_t* __restrict__ posB, const uint16_t* __restrict__ jB,
                 uint32_t* __restrict__ slotB, float* __restrict__ w_ent, int64_t w_cap,
                 Slot* __restrict__ slots, uint64_t mask, uint64_t home_base, uint64_t home_m,
                 int home_shr, int init_type, float init_v, float init_s, uint64_t seed,
                 int32_t* __restrict__ err, int32_t* __restrict__ inserted, UpdateParams p,
                 double* __restrict__ stats, int acc_stripes, uint32_t* __restrict__ hist,
                 int nbins, int hist_stripes, double* __restrict__ metrics,
                 int64_t* __restrict__ step_counter) {
  using namespace tpf;
  using namespace tpf2;
  __shared__ long long acc[2 * kUnitK];  // fixed-point sums of both units; then B weights
  __shared__ uint32_t smax[2];
  float* wj = reinterpret_cast<float*>(acc);
  const int t = threadIdx.x, b = blockIdx.x, lane = t & 63;
  if (do_upd && hist && b == (int)gridDim.x - 1) {  // (an extra workgroup, as tpf_step_kernel)
    auc_hist_block(hist, nbins, hist_stripes, metrics, step_counter);
    return;
  }
  // per-unit counts (clamped to the regions: a corrupted count never leaves them)
  int DA0 = 0, DA1 = 0, EA0 = 0, EA = 0, DB0 = 0, DB1 = 0, EB0 = 0, EB = 0;
  if (do_upd) {
    const int32_t* c = cntA + (int64_t)b * 4;
    EA0 = min(max(c[1], 0), kEC);
    DA0 = max(min(c[0], kUnitK), 0);
    DA1 = max(min(c[2], kUnitK), 0);
    EA = EA0 + max(min(c[3], kEC - EA0), 0);
  }
  if (do_res) {
    const int32_t* c = cntB + (int64_t)b * 4;
    EB0 = min(max(c[1], 0), kEC);
    DB0 = max(min(c[0], kUnitK), 0);
    DB1 = max(min(c[2], kUnitK), 0);
    EB = EB0 + max(min(c[3], kEC - EB0), 0);
  }
  const int DA = DA0 + DA1, DB = DB0 + DB1;
  const int64_t ebase = (int64_t)b * kEC, kbase = (int64_t)b * kUC;
  // key q of the flat index space -> its slot in the key region (unit 1 after unit 0)
  auto kreg = [&](int q, int D0) -> int64_t {
    return kbase + (q < D0 ? q : kUnitK + (q - D0));
  };
  auto kacc = [&](int q, int D0) -> int { return q < D0 ? q : kUnitK + (q - D0); };
  // ---- prefetch: A entries' partials, A keys' slot records, B keys' probes, B entries
  float v[kRE];
  uint16_t ja[kRE];
  float vmax0 = 0.f, vmax1 = 0.f;
  // (loads in batches at clamped in-region addresses, selects afterwards: a guarded load
  // per element compiles to a branch + s_waitcnt each)
  // (A's arrays are null on a pull-only launch: every A load is under do_upd)
  uint32_t sa[kRS];
  Slot sl[kRS];
#pragma unroll
  for (int r = 0; r < kRE; ++r) {
    v[r] = 0.f;
    ja[r] = 0;
  }
#pragma unroll
  for (int i = 0; i < kRS; ++i) sa[i] = kNoSlot;
  if (do_upd) {
    int32_t pa[kRE];
#pragma unroll
    for (int r = 0; r < kRE; ++r) {
      const int g = r * kThr + t;
      const int64_t gi = ebase + (g < EA ? g : 0);
      pa[r] = posA[gi];
      ja[r] = jA[gi];
    }
#pragma unroll
    for (int r = 0; r < kRE; ++r) {
      const bool ok = r * kThr + t < EA && in_range(pa[r], p_cap);
      const float x = psum[ok ? pa[r] : 0];
      v[r] = ok ? x : 0.f;
      if (r * kThr + t >= EA) ja[r] = 0;
    }
#pragma unroll
    for (int i = 0; i < kRS; ++i) {
      const int q = i * kThr + t;
      const uint32_t si = slotA[q < DA ? kreg(q, DA0) : kbase];
      sa[i] = (q < DA && si != kNoSlot && si <= mask) ? si : kNoSlot;
    }
#pragma unroll
    for (int i = 0; i < kRS; ++i) sl[i] = slots[sa[i] != kNoSlot ? sa[i] : 0];
  }
  uint32_t sb[kRP];
  float wb[kRP];
  bool fresh[kRP];
  int ins = 0;
#pragma unroll
  for (int i = 0; i < kRP; ++i) {
    const int q = i * kThr + t;
    sb[i] = kNoSlot;
    wb[i] = 0.f;
    fresh[i] = false;
    if (q < DB) {
      const int ins0 = ins;
      sb[i] = tpf_resolve(slots, mask, home_base, home_m, home_shr, uniqB[kreg(q, DB0)],
                          init_type, init_v, init_s, seed, &wb[i], &ins);
      fresh[i] = ins != ins0;  // inserted now: not in A, its weight is final
      if (sb[i] == kNoSlot && err) atomicOr(err, 1);  // table full
      slotB[kreg(q, DB0)] = sb[i];
    }
  }
  int32_t pb[kRB];
  uint16_t jb[kRB];
#pragma unroll
  for (int r = 0; r < kRB; ++r) {
    const int g = r * kThr + t;
    pb[r] = -1;
    jb[r] = 0;
    if (g < EB) {
      pb[r] = posB[ebase + g];
      jb[r] = jB[ebase + g];
    }
  }
  double dnnz = 0, wsum = 0, dsum = 0;
  if (do_upd) {
    for (int q = t; q < DA; q += kThr) acc[kacc(q, DA0)] = 0ll;
    if (t < 2) smax[t] = 0u;
#pragma unroll
    for (int r = 0; r < kRE; ++r) {
      const int g = r * kThr + t;
      if (g < EA0) vmax0 = fmaxf(vmax0, fabsf(v[r]));
      else vmax1 = fmaxf(vmax1, fabsf(v[r]));
    }
    for (int g = kRE * kThr + t; g < EA; g += kThr) {  // (rare: > 2048 entries)
      const int32_t pos = posA[ebase + g];
      const float x = in_range(pos, p_cap) ? fabsf(psum[pos]) : 0.f;
      if (g < EA0) vmax0 = fmaxf(vmax0, x);
      else vmax1 = fmaxf(vmax1, x);
    }
    __syncthreads();  // acc / smax zeroed
    fx_tile_max(vmax0, &smax[0]);
    fx_tile_max(vmax1, &smax[1]);
    __syncthreads();
    const int k20 = fx_shift(smax[0]), k21 = fx_shift(smax[1]);
    const double sc0 = ldexp(1.0, k20), sc1 = ldexp(1.0, k21);
#pragma unroll
    for (int r = 0; r < kRE; ++r) {
      const int g = r * kThr + t;
      if (g < EA && v[r] != 0.f && ja[r] < kUnitK) {
        const bool u1 = g >= EA0;
        fx_add(acc, (u1 ? kUnitK : 0) + ja[r], v[r], u1 ? sc1 : sc0);
      }
    }
    for (int g = kRE * kThr + t; g < EA; g += kThr) {
      const int32_t pos = posA[ebase + g];
      const uint16_t j = jA[ebase + g];
      const float x = in_range(pos, p_cap) ? psum[pos] : 0.f;
      const bool u1 = g >= EA0;
      if (x != 0.f && j < kUnitK) fx_add(acc, (u1 ? kUnitK : 0) + j, x, u1 ? sc1 : sc0);
    }
    __syncthreads();
    const double isc0 = ldexp(1.0, -k20), isc1 = ldexp(1.0, -k21);
    auto upd = [&](int q, Slot& s_, uint32_t si) {
      const double isc = q < DA0 ? isc0 : isc1;
      const float gs = (float)((double)acc[kacc(q, DA0)] * isc) * p.grad_scale;
      if (gs != gs) return;
      const float w_old = apply_update(s_, gs, p);
      slots[si] = s_;
      dnnz += (double)((s_.w != 0.f) - (w_old != 0.f));
      wsum += (double)s_.w * s_.w;
      const double d = (double)s_.w - w_old;
      dsum += d * d;
    };
#pragma unroll
    for (int i = 0; i < kRS; ++i)
      if (sa[i] != kNoSlot) upd(i * kThr + t, sl[i], sa[i]);
    for (int q = kRS * kThr + t; q < DA; q += kThr) {  // (rare: > 512 keys)
      const uint32_t si = slotA[kreg(q, DA0)];
      if (si == kNoSlot || si > mask) continue;
      Slot s_ = slots[si];
      upd(q, s_, si);
    }
    __syncthreads();  // (the updated records are what B re-reads; acc is free for wj)
  }
  if (do_res) {
#pragma unroll
    for (int i = 0; i < kRP; ++i) {
      const int q = i * kThr + t;
      if (q >= DB) continue;
      float w = wb[i];
      // a key that existed may have been updated by A just now: its weight again
      if (do_upd && !fresh[i] && sb[i] != kNoSlot) w = slots[sb[i]].w;
      wj[kacc(q, DB0)] = w;
    }
    for (int q = kRP * kThr + t; q < DB; q += kThr) {  // (rare: > 1024 keys)
      float w;
      const uint32_t si = tpf_resolve(slots, mask, home_base, home_m, home_shr,
                                      uniqB[kreg(q, DB0)], init_type, init_v, init_s, seed, &w,
                                      &ins);
      if (si == kNoSlot && err) atomicOr(err, 1);
      slotB[kreg(q, DB0)] = si;
      wj[kacc(q, DB0)] = w;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRB; ++r) {
      const int g = r * kThr + t;
      if (g < EB && in_range(pb[r], w_cap) && jb[r] < kUnitK)
        w_ent[pb[r]] = wj[(g >= EB0 ? kUnitK : 0) + jb[r]];
    }
    for (int g = kRB * kThr + t; g < EB; g += kThr) {
      const int32_t pos = posB[ebase + g];
      const uint16_t j = jB[ebase + g];
      if (in_range(pos, w_cap) && j < kUnitK) w_ent[pos] = wj[(g >= EB0 ? kUnitK : 0) + j];
    }
  }
  if (do_upd && stats) {
    const double a = wave_sum_dpp(dnnz), bb = wave_sum_dpp(wsum), cc = wave_sum_dpp(dsum);
    if (lane == 63) {
      double* st = acc_stripe(stats, acc_stripes);
      if (a != 0) atomicAdd(&st[0], a);
      if (bb != 0) atomicAdd(&st[1], bb);
      if (cc != 0) atomicAdd(&st[2], cc);
    }
  }
  if (inserted) {
    const int tot = wave_sum(ins);
    if (lane == 0 && tot) atomicAdd(inserted, tot);
  }
}

// ---- the padded multi-GPU exchange on the flat layout (G peers, G a power of two that
// divides the bucket workgroups: owner p's key range is exactly the buckets
// [p * B / G, (p + 1) * B / G), whose keys are rank-sorted (tpf_bucket sorted = 1), so
// the rows stay key-ordered for the owner's partitioned apply). A bucket's keys sit in
// its owner's row after those of the owner's earlier buckets: that offset is the sum of
// < B / G earlier counts, read straight from cnt[] (the bucket kernel has completed),
// so no bucket waits for another.
__device__ __forceinline__ int tpf_row_base(const int32_t* __restrict__ cnt, int b, int per,
                                            uint32_t* red /* LDS [kThr/64 + 1] */) {
  const int b0 = (b / per) * per;
  int s = 0;
  for (int q = b0 + (int)threadIdx.x; q < b; q += blockDim.x) s += cnt[4 * q] + cnt[4 * q + 2];
  uint32_t tot;
  tp_block_scan<tpf::kThr>((uint32_t)s, red, &tot);
  return (int)tot;
}

// keys of every bucket into its owner's row of `send` ([nkeys, ngrads, -, - | keys (C x kw
// words) | grads]); the owner's last bucket writes the row's key count; keys past C
// count as overflow (ovf, once per owner)
// (the key of unit-concatenated index i of bucket b)
__device__ __forceinline__ uint64_t tpf_key_at(const uint64_t* __restrict__ uniqf, int b, int D0,
                                               int i) {
  return i < D0 ? uniqf[(int64_t)b * tpf::kUC + i]
                : uniqf[(int64_t)b * tpf::kUC + tpf::kUnitK + (i - D0)];
}

// homes != null (the merged exchange): the row also carries, at word b0, the bounds of
// the owner's 2^lgP key-range partitions over the row's sorted keys (bnd[q] = # keys of
// partitions < q, bnd[P] = row count) -- what the owner's one-launch resolve + apply
// (kv_owner_part) needs to find its partition's run in every row. homes[2p], [2p+1] =
// owner p's ordered-home (base, m) (kv_slot.cuh key_part).
__global__ void __launch_bounds__(tpf::kThr)
tpf_pack_keys_kernel(const int32_t* __restrict__ cnt, const uint64_t* __restrict__ uniqf, int per,
                     int64_t C, int kw, int64_t H, int32_t* __restrict__ send,
                     int32_t* __restrict__ ovf, const uint64_t* __restrict__ homes, int64_t b0,
                     int lgP) {
  using namespace tpf;
  __shared__ uint32_t red[kThr / 64 + 1];
  const int b = blockIdx.x, p = b / per, t = threadIdx.x;
  const int base = tpf_row_base(cnt, b, per, red);
  const int D0 = min(cnt[4 * b], kUnitK), D1 = min(cnt[4 * b + 2], kUnitK);
  int32_t* row = send + (int64_t)p * H;
  const int P = 1 << lgP;
  const uint64_t hb = homes ? homes[2 * p] : 0, hm = homes ? homes[2 * p + 1] : 0;
  int32_t* rb = row + b0;
  // the key before this bucket's first one in the row: the last key of the nearest
  // non-empty earlier bucket of the same owner (none: the row's first key)
  int qprev = -1;
  if (homes && base > 0 && t == 0) {
    for (int c = b - 1; c >= (b / per) * per; --c) {
      const int e0 = min(cnt[4 * c], kUnitK), e1 = min(cnt[4 * c + 2], kUnitK);
      if (e0 + e1 > 0) {
        qprev = key_part(tpf_key_at(uniqf, c, e0, e0 + e1 - 1), hb, hm, lgP);
        break;
      }
    }
  }
  if (homes) {  // (broadcast qprev through the scan scratch)
    __syncthreads();
    if (t == 0) red[0] = (uint32_t)(qprev + 1);
    __syncthreads();
    qprev = (int)red[0] - 1;
  }
  for (int i = t; i < D0 + D1; i += kThr) {
    const int64_t pos = (int64_t)base + i;
    if (pos >= C) break;
    const uint64_t k = tpf_key_at(uniqf, b, D0, i);
    if (kw == 1) row[4 + pos] = (int32_t)(uint32_t)k;
    else reinterpret_cast<uint64_t*>(row + 4)[pos] = k;
    if (homes) {
      const int q = key_part(k, hb, hm, lgP);
      const int q0 = (i > 0 ? key_part(tpf_key_at(uniqf, b, D0, i - 1), hb, hm, lgP) : qprev) + 1;
      for (int j = q0; j <= q; ++j) rb[j] = (int32_t)pos;
      if (pos == C - 1)  // a full row ends here
        for (int j = q + 1; j <= P; ++j) rb[j] = (int32_t)C;
    }
  }
  if (t == 0 && b % per == per - 1) {
    const int64_t tot = (int64_t)base + D0 + D1;
    row[0] = (int32_t)(tot < C ? tot : C);
    if (tot > C && ovf) atomicAdd(ovf, (int32_t)(tot - C));
    if (homes && tot <= C) {  // the row's tail bounds after its last key
      int qlast = -1;
      for (int c = b; c >= (b / per) * per; --c) {
        const int e0 = min(cnt[4 * c], kUnitK), e1 = min(cnt[4 * c + 2], kUnitK);
        if (e0 + e1 > 0) {
          qlast = key_part(tpf_key_at(uniqf, c, e0, e0 + e1 - 1), hb, hm, lgP);
          break;
        }
      }
      for (int j = qlast + 1; j <= P; ++j) rb[j] = (int32_t)tot;
    }
  }
}

// pulled weights (row order, wrecv[p * C + i]) -> LDS per unit key -> the bucket's
// entries in tile-entry order (w_ent) for the flat fused forward
__global__ void __launch_bounds__(tpf::kThr)
tpf_unpack_w_kernel(const int32_t* __restrict__ cnt, const int32_t* __restrict__ ent_pos,
                    const uint16_t* __restrict__ ent_j, int per, int64_t C,
                    const float* __restrict__ wrecv, int64_t wstride, float* __restrict__ w_ent,
                    int64_t w_cap) {
  using namespace tpf;
  __shared__ uint32_t red[kThr / 64 + 1];
  __shared__ float wj[kUnitK];
  const int b = blockIdx.x, p = b / per, t = threadIdx.x;
  const int base = tpf_row_base(cnt, b, per, red);
  const int32_t* c = cnt + 4 * b;
  int off = base;
#pragma unroll 1
  for (int s = 0; s < 2; ++s) {
    const int e0 = s ? min(max(c[1], 0), kEC) : 0;
    const int D = min(c[2 * s], kUnitK), E = min(c[2 * s + 1], kEC - e0);
    if (D <= 0) continue;
    for (int j = t; j < D; j += kThr) {
      const int64_t pos = (int64_t)off + j;
      wj[j] = pos < C ? wrecv[(int64_t)p * wstride + pos] : 0.f;
    }
    __syncthreads();
    const int64_t eb = (int64_t)b * kEC + e0, rb = (int64_t)b * kEC;
    for (int g0 = 0; g0 < E; g0 += 8 * kThr) {  // (8 entries per thread: loads batched)
      int32_t pp[8];
      uint16_t jq[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int g = g0 + q * kThr + t;
        const int64_t gi = g < E ? eb + g : rb;
        pp[q] = ent_pos[gi];
        jq[q] = ent_j[gi];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (g0 + q * kThr + t < E && in_range(pp[q], w_cap) && jq[q] < kUnitK)
          w_ent[pp[q]] = wj[jq[q]];
    }
    __syncthreads();
    off += D;
  }
}

// every key's gradient (its entries' partials summed in LDS, 64-bit fixed point as in
// tpf_step) into its owner's row; ff = 1: f32 into gstage[p * C + i] and the row's
// FixingFloat min / max (header words 2 / 3, order-preserving ints; xchg_ff_init ran
// first) for xchg_ff_encode. The owner's last bucket writes the row's gradient count.
// Block 0: the step's AUC epilogue and the overflow flag to the host.
__device__ __forceinline__ int tpf_ff_ord(float f) {
  const int b = __float_as_int(f);
  return b >= 0 ? b : b ^ 0x7fffffff;
}
__global__ void __launch_bounds__(tpf::kThr)
tpf_pack_grads_kernel(const int32_t* __restrict__ cnt, const int32_t* __restrict__ ent_pos,
                      const uint16_t* __restrict__ ent_j, int per, int64_t C, int kw, int64_t H,
                      const float* __restrict__ psum, int64_t p_cap, int32_t* __restrict__ send,
                      int ff, float* __restrict__ gstage, uint32_t* __restrict__ hist,
                      int hist_stripes, double* __restrict__ metrics,
                      int64_t* __restrict__ step_counter, const int32_t* __restrict__ ovf,
                      int32_t* __restrict__ ovf_host) {
  using namespace tpf;
  __shared__ uint32_t red[kThr / 64 + 1];
  __shared__ long long acc[kUnitK];
  __shared__ uint32_t smax;
  const int b = blockIdx.x, p = b / per, t = threadIdx.x, lane = t & 63;
  if ((hist || ovf_host) && b == (int)gridDim.x - 1) {  // extra workgroup (the launcher adds it)
    if (ovf_host && t == 0) ovf_host[0] = ovf[0];
    if (hist) auc_hist_block(hist, 2048, hist_stripes, metrics, step_counter);
    return;
  }
  const int base = tpf_row_base(cnt, b, per, red);
  const int32_t* c = cnt + 4 * b;
  int32_t* row = send + (int64_t)p * H;
  float* grow = reinterpret_cast<float*>(row + 4 + C * kw);
  float lo = 3.4e38f, hi = -3.4e38f;
  int off = base;
#pragma unroll 1
  for (int s = 0; s < 2; ++s) {
    const int e0 = s ? min(max(c[1], 0), kEC) : 0;
    const int D = min(c[2 * s], kUnitK), E = min(c[2 * s + 1], kEC - e0);
    if (D <= 0) continue;
    const int64_t eb = (int64_t)b * kEC + e0;
    for (int j = t; j < D; j += kThr) acc[j] = 0ll;
    if (t == 0) smax = 0u;
    float vmax = 0.f;
    // the first 2048 entries' (pos, j) and partials in registers, loaded in two batches
    // at clamped in-region addresses (a guarded dependent load pair per entry compiled
    // to serialised round trips); the rest (rare) in a loop
    constexpr int kR = 8;
    const int64_t rb = (int64_t)b * kEC;
    int32_t pr[kR];
    uint16_t jr[kR];
    float xr[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const int g = r * kThr + t;
      const int64_t gi = g < E ? eb + g : rb;
      pr[r] = ent_pos[gi];
      jr[r] = ent_j[gi];
    }
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const bool ok = r * kThr + t < E && in_range(pr[r], p_cap);
      const float x = psum[ok ? pr[r] : 0];
      xr[r] = ok ? x : 0.f;
      vmax = fmaxf(vmax, fabsf(xr[r]));
    }
    for (int g = kR * kThr + t; g < E; g += kThr) {
      const int32_t pos = ent_pos[eb + g];
      if (in_range(pos, p_cap)) vmax = fmaxf(vmax, fabsf(psum[pos]));
    }
    __syncthreads();
    fx_tile_max(vmax, &smax);
    __syncthreads();
    const int k2 = fx_shift(smax);
    const double sc = ldexp(1.0, k2);
#pragma unroll
    for (int r = 0; r < kR; ++r)
      if (xr[r] != 0.f && jr[r] < kUnitK) fx_add(acc, jr[r], xr[r], sc);
    for (int g = kR * kThr + t; g < E; g += kThr) {
      const int32_t pos = ent_pos[eb + g];
      const uint16_t j = ent_j[eb + g];
      const float x = in_range(pos, p_cap) ? psum[pos] : 0.f;
      if (x != 0.f && j < kUnitK) fx_add(acc, j, x, sc);
    }
    __syncthreads();
    const double isc = ldexp(1.0, -k2);
    for (int j = t; j < D; j += kThr) {
      const int64_t pos = (int64_t)off + j;
      if (pos >= C) break;
      const float g = (float)((double)acc[j] * isc);
      if (ff) {
        gstage[(int64_t)p * C + pos] = g;
        if (g == g) {
          lo = fminf(lo, g);
          hi = fmaxf(hi, g);
        }
      } else {
        grow[pos] = g;
      }
    }
    __syncthreads();  // (acc of the next unit)
    off += D;
  }
  if (ff) {
    // the workgroup's min / max -> its partial at gstage[G * C + 2 b] (xchg_ff_encode
    // reduces a row's partials): per-wave atomics on the row header's two words were
    // ~8 k device-scope atomics on 16 addresses per step, serialised across the XCDs
    // (pack 16 -> 32 us with fixing-float at 8 emulated peers, gpurun r6u)
    lo = wave_min(lo);
    hi = wave_max(hi);
    __shared__ float sl[kThr / 64], sh[kThr / 64];
    if (lane == 0) {
      sl[t >> 6] = lo;
      sh[t >> 6] = hi;
    }
    __syncthreads();
    if (t == 0) {
      for (int w = 1; w < kThr / 64; ++w) {
        lo = fminf(lo, sl[w]);
        hi = fmaxf(hi, sh[w]);
      }
      float* part = gstage + (int64_t)(gridDim.x - ((hist || ovf_host) ? 1 : 0)) / per * C;
      part[2 * b] = lo;
      part[2 * b + 1] = hi;
    }
  }
  if (t == 0 && b % per == per - 1) row[1] = (int32_t)(off < C ? off : C);
}

// ---------------------------------------------------------------------------
struct TpGeom {
  int nbk, shift;
  int lts;      // log2 occurrences per tile
  int64_t T, N;  // tiles, entry stride (T * kTile)
};

// Occurrences per tile of the FLAT layout, 2^lts in [1024, 8192]: the largest that still
// gives >= 128 tiles, so a small minibatch (B = 10,000 x 39: 48 tiles of 8192, i.e. 48
// busy CUs, each tile's LDS insert chain ~15 us) spreads over the chip; large ones keep
// 8192 (fewer tiles = fewer tile entries of the hot keys). Measured at B = 10,000
// (profiles/r5_adaptive_tiles.log): 8192 -> 260.6 M ex/s, 4096 -> 304.3, 2048 -> 309.3,
// 1024 -> 196.8 (the hot keys' extra entries). Entry ids keep the kTile stride whatever
// the tile holds. The compact "tp" layout always uses 8192.
// PSAMD_TILE_LTS=10..13 pins it (A/B), PSAMD_TILE_MIN the tile target.
static int tp_flat_lts(int64_t n) {
  // (read per call: host-side geometry only, a few calls per launch list build)
  const char* pe = getenv("PSAMD_TILE_LTS");
  const int pin = pe ? atoi(pe) : 0;
  const char* te = getenv("PSAMD_TILE_MIN");
  int tmin = te ? atoi(te) : 128;
  tmin = tmin < 1 ? 1 : tmin > tp::kMaxT / 2 ? tp::kMaxT / 2 : tmin;
  int lts = 13;
  if (pin >= 10 && pin <= 13) {
    lts = pin;
  } else {
    while (lts > 10 && ((n + (1ll << lts) - 1) >> lts) < tmin) --lts;
  }
  while (lts < 13 && ((n + (1ll << lts) - 1) >> lts) > tp::kMaxT) ++lts;  // (LDS tile runs)
  return lts;
}

static TpGeom tp_geom(int64_t n, int bits, bool flat = false) {
  TpGeom g;
  g.lts = flat ? tp_flat_lts(n) : 13;
  static_assert(tp::kTile == 8192, "tile entry stride 2^13");
  g.T = (n + (1ll << g.lts) - 1) >> g.lts;
  g.N = g.T * tp::kTile;
  // <= 1024 occurrences per bucket on average: even if every key is distinct a PAIR of
  // buckets (the flat layout's unit) stays under the kDH-key hash (at 1280, nearly
  // distinct minibatches -- e.g. 1000 rcv1-width rows over 10^8 ids -- overflowed every
  // pair into the register-light fallback: ~20x slower bucket kernel). The 2048-bucket
  // cap leaves the Criteo-shaped 65,536 x 39 batch as before (measured there: <= 1615
  // entries and 157 distinct keys per bucket at 2048 buckets)
  int bb = 0;
  while (bb < 11 && (n >> bb) > 1024) ++bb;
  if (bb > bits) bb = bits;
  g.nbk = 1 << bb;
  g.shift = bits - bb;
  return g;
}

int64_t tploc_stride(int64_t n) { return tp_geom(n, 31).N; }
// flat layout: the entry stride of an n-key minibatch, and a bound over every minibatch of
// <= n keys (a workspace sized for n must take smaller minibatches, which may use more,
// smaller tiles): <= kMaxT tiles, and tiles of 1024 at the least
int64_t tpf_stride(int64_t n) { return tp_geom(n, 31, true).N; }
int64_t tpf_stride_max(int64_t n) {
  const int64_t t = std::min<int64_t>(tp::kMaxT, (n + 1023) / 1024);
  return std::max<int64_t>(t, (n + tp::kTile - 1) / tp::kTile) * tp::kTile;
}
int tpf_tile_log2(int64_t n) { return tp_geom(n, 31, true).lts; }
int tploc_buckets(int64_t n, int bits) { return tp_geom(n, bits).nbk; }
int tploc_tile() { return tp::kTile; }

bool tploc_supported(int64_t n, int bits) {
  // <= 34 bits: quotient-encoded tile hash; bucket suffixes (bits - log2 nbk) < 32 bits
  return bits >= 2 && bits <= 34 && n > 0 && (n >> 11) <= 1280 &&
         (n + tp::kTile - 1) / tp::kTile <= tp::kMaxT && tp_geom(n, bits).shift <= 31;
}

static size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

size_t tploc_temp_bytes(int64_t n, int bits) {
  const TpGeom g = tp_geom(n, bits);
  return al16((size_t)g.nbk * 8 + 16)                          // look-back status + epoch
         + al16((size_t)g.N * 4)                               // tkeys
         + al16((size_t)g.T * (g.nbk + 1) * 2);                // toff (u16)
}

// temp's first (nbk * 8 + 16) bytes (status words + epoch) must be zero before the
// first launch (the Python side allocates it zeroed); they need no reset afterwards
void localize_tp(const uint64_t* raw, int64_t n, KeyMix m, void* temp, size_t temp_bytes,
                 int32_t* dcnt, uint16_t* rep, int32_t* pos_s, int32_t* segid, uint64_t* uniq,
                 int32_t* seg_start, int32_t* ent_uid, int32_t* local_col, int32_t* n_uniq,
                 int32_t* n_ent, float* grad, unsigned long long* pieces, int32_t* err,
                 int64_t u_cap, uint64_t* prof, hipStream_t st) {
  if (n <= 0) return;
  if (!tploc_supported(n, m.bits)) throw std::runtime_error("localize_tp: unsupported size");
  if (temp_bytes < tploc_temp_bytes(n, m.bits)) throw std::runtime_error("localize_tp: temp");
  const TpGeom g = tp_geom(n, m.bits);
  char* p = (char*)temp;
  auto take = [&](size_t bytes) { char* r = p; p += al16(bytes); return r; };
  uint64_t* status = (uint64_t*)take((size_t)g.nbk * 8 + 16);
  uint32_t* epoch = (uint32_t*)(status + g.nbk);
  uint32_t* tkeys = (uint32_t*)take((size_t)g.N * 4);
  uint16_t* toff = (uint16_t*)take((size_t)g.T * (g.nbk + 1) * 2);
  static const char* quot_env = getenv("PSAMD_TP_QUOT");  // "1": A/B the encoding at <= 31 bits
  if (m.bits > 31 || (quot_env && quot_env[0] == '1'))
    tp_tile_kernel<true><<<(unsigned)g.T, tp::kThr, 0, st>>>(raw, n, m, g.shift, g.nbk, tkeys, toff,
                                                             dcnt, rep, err, g.lts);
  else
    tp_tile_kernel<false><<<(unsigned)g.T, tp::kThr, 0, st>>>(raw, n, m, g.shift, g.nbk, tkeys, toff,
                                                              dcnt, rep, err, g.lts);
  PSAMD_HIP_CHECK(hipGetLastError());
  // buckets in pairs of fine buckets: one round of workgroups (the pair's key bit above
  // a <= 30-bit suffix keeps the LDS hash's empty word unreachable)
  const bool pair = g.nbk >= 2 && g.shift <= 30;
  tp_bucket_kernel<<<(unsigned)(pair ? g.nbk / 2 : g.nbk), tp::kBkThr, 0, st>>>(
      tkeys, toff, g.nbk, pair ? 1 : 0, (int)g.T, g.shift, status, epoch, pos_s, segid, uniq,
      seg_start, ent_uid, n_uniq, n_ent, grad, pieces, u_cap, g.N, err, prof);
  PSAMD_HIP_CHECK(hipGetLastError());
  if (local_col) {  // (skipped when the fused forward reads the entry map directly)
    tp_gather_kernel<<<(unsigned)((n + 1023) / 1024), 256, 0, st>>>(rep, ent_uid, n, local_col);
    PSAMD_HIP_CHECK(hipGetLastError());
  }
}

// ---- flat (tpf) host side
// (PSAMD_TPF_PAIR=0: one fine bucket per workgroup -- measurement of the pair layout)
static bool tpf_pair(const TpGeom& g) {
  static const int force = [] {
    const char* e = std::getenv("PSAMD_TPF_PAIR");
    return e ? std::atoi(e) : -1;
  }();
  return g.nbk >= 2 && g.shift <= 30 && force != 0;
}
static int tpf_groups_of(const TpGeom& g) { return tpf_pair(g) ? g.nbk / 2 : g.nbk; }
int tpf_groups(int64_t n, int bits) { return tpf_groups_of(tp_geom(n, bits)); }
int tpf_key_region() { return tpf::kUC; }
int tpf_entry_region() { return tpf::kEC; }

size_t tpf_temp_bytes(int64_t n, int bits) {  // (any minibatch of <= n keys: tpf_stride_max)
  const int64_t N = tpf_stride_max(n);
  return al16((size_t)N * 4) + al16((size_t)(N / tp::kTile) * (tp::kMaxBk + 1) * 2);  // tkeys, toff
}

// uniqf >= groups * kUC, ent_pos / ent_j >= groups * kEC, cnt >= groups * 4 (the host
// checks; tpf_groups)
// Tail filter (filt != null): ecnt >= tpf_stride_max(n) bytes, w_ent >= w_cap floats, and
// the sketch's regions no coarser than a fine bucket (region = key >> rshift, rshift <=
// shift; the host checks).
void localize_tpf(const uint64_t* raw, int64_t n, KeyMix m, void* temp, size_t temp_bytes,
                  int32_t* dcnt, uint16_t* rep, uint64_t* uniqf, int32_t* ent_pos, uint16_t* ent_j,
                  int32_t* cnt, int32_t* err, bool sorted, hipStream_t st, const CmArgs* filt,
                  uint8_t* ecnt, float* w_ent, int64_t w_cap, int32_t* cnt_pre, int stage) {
  if (n <= 0) return;
  if (!tploc_supported(n, m.bits)) throw std::runtime_error("localize_tpf: unsupported size");
  if (temp_bytes < tpf_temp_bytes(n, m.bits)) throw std::runtime_error("localize_tpf: temp");
  const TpGeom g = tp_geom(n, m.bits, true);
  if (filt && (filt->rshift > g.shift || !ecnt || !w_ent))
    throw std::runtime_error("localize_tpf: tail filter regions coarser than a bucket");
  char* p = (char*)temp;
  auto take = [&](size_t bytes) { char* r = p; p += al16(bytes); return r; };
  uint32_t* tkeys = (uint32_t*)take((size_t)g.N * 4);
  uint16_t* toff = (uint16_t*)take((size_t)g.T * (g.nbk + 1) * 2);
  // stage 1: the tile kernel only, 2: the bucket kernel only, 3: (tail filter) the filter
  // kernel only, 4: tile + bucket -- a caller orders something between them (the tail
  // filter's filter kernels run in minibatch order); 0: all
  const bool q = m.bits > 31;
  if (stage == 2) goto bucket;
  if (stage == 3) goto filter;
  if (filt && q)
    tp_tile_kernel<true, true><<<(unsigned)g.T, tp::kThr, 0, st>>>(
        raw, n, m, g.shift, g.nbk, tkeys, toff, dcnt, rep, err, g.lts, ecnt);
  else if (filt)
    tp_tile_kernel<false, true><<<(unsigned)g.T, tp::kThr, 0, st>>>(
        raw, n, m, g.shift, g.nbk, tkeys, toff, dcnt, rep, err, g.lts, ecnt);
  else if (q)
    tp_tile_kernel<true><<<(unsigned)g.T, tp::kThr, 0, st>>>(raw, n, m, g.shift, g.nbk, tkeys, toff,
                                                             dcnt, rep, err, g.lts);
  else
    tp_tile_kernel<false><<<(unsigned)g.T, tp::kThr, 0, st>>>(raw, n, m, g.shift, g.nbk, tkeys, toff,
                                                              dcnt, rep, err, g.lts);
  PSAMD_HIP_CHECK(hipGetLastError());
  if (stage == 1) return;
bucket : {
  const int pair = tpf_pair(g) ? 1 : 0;
  if (filt)
    tpf_bucket_kernel<true><<<(unsigned)tpf_groups_of(g), tp::kBkThr, 0, st>>>(
        tkeys, toff, g.nbk, pair, (int)g.T, g.shift, uniqf, ent_pos, ent_j, cnt, err,
        sorted ? 1 : 0, ecnt);
  else
    tpf_bucket_kernel<false><<<(unsigned)tpf_groups_of(g), tp::kBkThr, 0, st>>>(
        tkeys, toff, g.nbk, pair, (int)g.T, g.shift, uniqf, ent_pos, ent_j, cnt, err,
        sorted ? 1 : 0, nullptr);
  PSAMD_HIP_CHECK(hipGetLastError());
}
  if (stage == 2 || stage == 4 || !filt) return;
filter:
  if (!filt) return;
  tpf_filter_kernel<<<(unsigned)tpf_groups_of(g), tp::kBkThr, 0, st>>>(
      uniqf, ent_pos, ent_j, cnt, ecnt, *filt, w_ent, w_cap, cnt_pre);
  PSAMD_HIP_CHECK(hipGetLastError());
}

// multi-GPU flat exchange: the owner of bucket workgroup b is b / per, per = groups / G
bool tpf_exchange_ok(int64_t n, int bits, int G) {
  const int groups = tpf_groups(n, bits);
  return G >= 1 && !(G & (G - 1)) && groups % G == 0;
}
static int tpf_per_owner(int64_t n, int bits, int G) {
  if (!tpf_exchange_ok(n, bits, G))
    throw std::runtime_error("tpf exchange: G must be a power of two dividing the bucket groups");
  return tpf_groups(n, bits) / G;
}

void tpf_pack_keys(int64_t n, int bits, int G, const int32_t* cnt, const uint64_t* uniqf, int64_t C,
                   int kw, int64_t H, int32_t* send, int32_t* ovf, const uint64_t* homes,
                   int64_t b0, int lgP, hipStream_t st) {
  const int per = tpf_per_owner(n, bits, G);
  tpf_pack_keys_kernel<<<(unsigned)tpf_groups(n, bits), tpf::kThr, 0, st>>>(
      cnt, uniqf, per, C, kw, H, send, ovf, homes, b0, lgP);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void tpf_unpack_w(int64_t n, int bits, int G, const int32_t* cnt, const int32_t* ent_pos,
                  const uint16_t* ent_j, int64_t C, const float* wrecv, int64_t wstride,
                  float* w_ent, int64_t w_cap, hipStream_t st) {
  const int per = tpf_per_owner(n, bits, G);
  tpf_unpack_w_kernel<<<(unsigned)tpf_groups(n, bits), tpf::kThr, 0, st>>>(
      cnt, ent_pos, ent_j, per, C, wrecv, wstride > 0 ? wstride : C, w_ent, w_cap);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void tpf_pack_grads(int64_t n, int bits, int G, const int32_t* cnt, const int32_t* ent_pos,
                    const uint16_t* ent_j, int64_t C, int kw, int64_t H, const float* psum,
                    int64_t p_cap, int32_t* send, bool ff, float* gstage, uint32_t* hist,
                    int hist_stripes, double* metrics, int64_t* step_counter, const int32_t* ovf,
                    int32_t* ovf_host, hipStream_t st) {
  const int per = tpf_per_owner(n, bits, G);
  // (+1 workgroup: the AUC epilogue / overflow publication, off unit 0's critical path)
  tpf_pack_grads_kernel<<<(unsigned)tpf_groups(n, bits) + ((hist || ovf_host) ? 1u : 0u),
                          tpf::kThr, 0, st>>>(
      cnt, ent_pos, ent_j, per, C, kw, H, psum, p_cap, send, ff ? 1 : 0, gstage, hist,
      hist_stripes, metrics, step_counter, ovf, ovf_host);
  PSAMD_HIP_CHECK(hipGetLastError());
}


// One launch of tpf_step_kernel over the groups of an n-key minibatch (A and B: the
// same n). A = null: pull only; B = null: update only.
void tpf_step(int64_t n, int bits, const int32_t* cntA, const int32_t* posA, const uint16_t* jA,
              const uint32_t* slotA, const float* psum, int64_t p_cap, const int32_t* cntB,
              const uint64_t* uniqB, const int32_t* posB, const uint16_t* jB, uint32_t* slotB,
              float* w_ent, int64_t w_cap, void* slots, int64_t cap, uint64_t home_base,
              uint64_t home_m, int init_type, float init_v, float init_s, uint64_t seed,
              int32_t* err, int32_t* inserted, int algo, int lr_type, float alpha, float beta,
              float l1, float l2, float grad_scale, float max_delta, double* stats,
              int acc_stripes, uint32_t* hist, int nbins, int hist_stripes, double* metrics,
              int64_t* step_counter, hipStream_t st) {
  if (n <= 0) return;
  if (hist && nbins != 2048) throw std::runtime_error("tpf_step: the fused AUC needs 2048 bins");
  if (cap > (int64_t)1 << 32) throw std::runtime_error("tpf_step: > 2^32 slots (u32 slot ids)");
  int lg = 0;
  while ((1ll << lg) < cap) ++lg;
  UpdateParams p{algo, lr_type, alpha, beta, l1, l2, grad_scale, max_delta};
  const int groups = tpf_groups(n, bits);
  // PSAMD_TPF_STEP2=1: the overlapped form (measured slower: 28.7-30.2 vs 24.9-25.4 us per
  // update + pull launch, profiles/r4_tpf_step_probe.log; kept for A/B and its test)
  const char* v2_env = getenv("PSAMD_TPF_STEP2");
  if (!(v2_env && v2_env[0] == '1'))
    tpf_step_kernel<<<(unsigned)groups + (cntA && hist ? 1u : 0u), tpf::kThr, 0, st>>>(
        cntA != nullptr, cntA, posA, jA, slotA, psum, p_cap, cntB != nullptr, cntB, uniqB, posB,
        jB, slotB, w_ent, w_cap, (Slot*)slots, (uint64_t)(cap - 1), home_base, home_m, 64 - lg,
        init_type, init_v, init_s, seed, err, inserted, p, stats, acc_stripes,
        cntA ? hist : nullptr, nbins, hist_stripes, metrics, step_counter);
  else
    tpf_step2_kernel<<<(unsigned)groups + (cntA && hist ? 1u : 0u), tpf::kThr, 0, st>>>(
        cntA != nullptr, cntA, posA, jA, slotA, psum, p_cap, cntB != nullptr, cntB, uniqB, posB,
        jB, slotB, w_ent, w_cap, (Slot*)slots, (uint64_t)(cap - 1), home_base, home_m, 64 - lg,
        init_type, init_v, init_s, seed, err, inserted, p, stats, acc_stripes,
        cntA ? hist : nullptr, nbins, hist_stripes, metrics, step_counter);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void tp_backward(const uint16_t* rep, const int32_t* dcnt, int64_t n, const int32_t* rows,
                 int width, const float* vals, const float* coef, int64_t B, float* psum,
                 const int32_t* pos_s, const int32_t* segid, const int32_t* n_ent, float* grad,
                 int64_t grad_cap, hipStream_t st) {
  if (n <= 0) return;
  const TpGeom g = tp_geom(n, 31);
  static const char* bwd_env = getenv("PSAMD_TP_BWD");  // "rows": A/B the row-major walk
  const bool cols = !(bwd_env && bwd_env[0] == 'r');
  if (cols && rows == nullptr && width >= 2 && width <= tp::kThr)
    tp_bwd_accum_cols_kernel<<<(unsigned)g.T, tp::kThr, 0, st>>>(rep, dcnt, n, width, vals, coef,
                                                                 B, psum);
  else
    tp_bwd_accum_kernel<<<(unsigned)g.T, tp::kThr, 0, st>>>(rep, dcnt, n, rows, width, vals, coef,
                                                            B, psum);
  PSAMD_HIP_CHECK(hipGetLastError());
  tp_seg_reduce_kernel<<<grid_for(g.N, 256, 2048), 256, 0, st>>>(pos_s, segid, g.N, n_ent, psum,
                                                                 g.N, grad, grad_cap);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void tp_gather(const uint16_t* rep, const int32_t* ent_uid, int64_t n, int32_t* local_col,
               hipStream_t st) {
  if (n <= 0) return;
  tp_gather_kernel<<<(unsigned)((n + 1023) / 1024), 256, 0, st>>>(rep, ent_uid, n, local_col);
  PSAMD_HIP_CHECK(hipGetLastError());
}

// register-held occurrences: PER = ceil(width / 8) in 2..8, NP = the row passes of
// the narrowest width with that PER (fewer register slots -> 2 workgroups per CU)
static int tp_fb_passes(int width) {
  return (int)((tp::kTile / width + 2 + tp::kThr / kFbLanes - 1) / (tp::kThr / kFbLanes));
}
static constexpr int kFbNP[9] = {0, 0, 8, 4, 3, 2, 2, 2, 2};

bool tp_fwd_bwd_supported(int width) {
  if (width < 9 || width > 64) return false;
  return tp_fb_passes(width) <= kFbNP[(width + kFbLanes - 1) / kFbLanes];
}

void tp_fwd_bwd(const uint16_t* rep, const int32_t* dcnt, const int32_t* ent_uid, int64_t n,
                int width, const float* vals, const float* w_local, int64_t w_cap,
                const float* labels, int64_t B, int loss_type, float* coef_out, double* metrics,
                uint32_t* hist, int nbins, int acc_stripes, int hist_stripes, float* psum,
                const int32_t* pos_s, const int32_t* segid, const int32_t* n_ent, float* grad,
                int64_t grad_cap, bool reduce, hipStream_t st) {
  if (n <= 0) return;
  if (!tp_fwd_bwd_supported(width) || n != B * (int64_t)width)
    throw std::runtime_error("tp_fwd_bwd: unsupported width or n != B * width");
  const bool flat = ent_uid == nullptr;  // w_local in tile-entry order (tpf)
  const TpGeom g = tp_geom(n, 31, flat);
  if (hist && (nbins <= 0 || nbins > kFbMaxBins))
    throw std::runtime_error("tp_fwd_bwd: 1..2048 AUC bins (LDS histogram)");
  const size_t lds = 0;
  const int per = (width + kFbLanes - 1) / kFbLanes;
  if (flat && w_cap < g.N) throw std::runtime_error("tp_fwd_bwd: flat w_ent < tile stride");
  // rows of one tile fit one register pass (<= 128 rows: 2^lts / width + 2): NP = 1
  const bool one = ((1 << g.lts) / width + 2) <= tp::kThr / kFbLanes;
#define PSAMD_FB(PER, NP)                                                                     \
  if (flat)                                                                                   \
    tp_fwd_bwd_kernel<PER, NP, true><<<(unsigned)g.T, tp::kThr, lds, st>>>(                  \
        rep, dcnt, ent_uid, n, width, vals, w_local, w_cap, labels, B, loss_type, coef_out,   \
        metrics, hist, nbins, acc_stripes, hist_stripes, psum, g.lts);                        \
  else                                                                                        \
    tp_fwd_bwd_kernel<PER, NP, false><<<(unsigned)g.T, tp::kThr, lds, st>>>(                 \
        rep, dcnt, ent_uid, n, width, vals, w_local, w_cap, labels, B, loss_type, coef_out,   \
        metrics, hist, nbins, acc_stripes, hist_stripes, psum, g.lts)
  if (one && flat) {
    switch (per) {
      case 2: PSAMD_FB(2, 1); break;
      case 3: PSAMD_FB(3, 1); break;
      case 4: PSAMD_FB(4, 1); break;
      case 5: PSAMD_FB(5, 1); break;
      case 6: PSAMD_FB(6, 1); break;
      case 7: PSAMD_FB(7, 1); break;
      default: PSAMD_FB(8, 1); break;
    }
  } else {
    switch (per) {  // NP = kFbNP[PER] row passes in registers (tp_fwd_bwd_supported)
      case 2: PSAMD_FB(2, 8); break;
      case 3: PSAMD_FB(3, 4); break;
      case 4: PSAMD_FB(4, 3); break;
      case 5: PSAMD_FB(5, 2); break;
      case 6: PSAMD_FB(6, 2); break;
      case 7: PSAMD_FB(7, 2); break;
      default: PSAMD_FB(8, 2); break;
    }
  }
#undef PSAMD_FB
  PSAMD_HIP_CHECK(hipGetLastError());
  if (!reduce) return;  // (the caller runs tp_seg_update instead)
  tp_seg_reduce_kernel<<<grid_for(g.N, 256, 2048), 256, 0, st>>>(pos_s, segid, g.N, n_ent, psum,
                                                                 g.N, grad, grad_cap);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void tp_fwd_bwd_csr(const uint16_t* rep, const int32_t* dcnt, const int32_t* ent_uid, int64_t n,
                    const int64_t* row_ptr, const int32_t* rows, const float* vals,
                    const float* w_local, int64_t w_cap, const float* labels, int64_t B,
                    int loss_type, float* coef_out, double* metrics, uint32_t* hist, int nbins,
                    int acc_stripes, int hist_stripes, float* psum, const int32_t* pos_s,
                    const int32_t* segid, const int32_t* n_ent, float* grad, int64_t grad_cap,
                    bool reduce, hipStream_t st) {
  if (n <= 0) return;
  const bool flat = ent_uid == nullptr;
  const TpGeom g = tp_geom(n, 31, flat);
  if (hist && (nbins <= 0 || nbins > kFbMaxBins))
    throw std::runtime_error("tp_fwd_bwd_csr: 1..2048 AUC bins (LDS histogram)");
  if (flat && w_cap < g.N) throw std::runtime_error("tp_fwd_bwd_csr: flat w_ent < tile stride");
  if (flat)
    tp_fwd_bwd_csr_kernel<true><<<(unsigned)g.T, tp::kThr, 0, st>>>(
        rep, dcnt, ent_uid, n, row_ptr, rows, vals, w_local, w_cap, labels, B, loss_type,
        coef_out, metrics, hist, nbins, acc_stripes, hist_stripes, psum, g.lts);
  else
    tp_fwd_bwd_csr_kernel<false><<<(unsigned)g.T, tp::kThr, 0, st>>>(
        rep, dcnt, ent_uid, n, row_ptr, rows, vals, w_local, w_cap, labels, B, loss_type,
        coef_out, metrics, hist, nbins, acc_stripes, hist_stripes, psum, g.lts);
  PSAMD_HIP_CHECK(hipGetLastError());
  if (!reduce) return;
  tp_seg_reduce_kernel<<<grid_for(g.N, 256, 2048), 256, 0, st>>>(pos_s, segid, g.N, n_ent, psum,
                                                                 g.N, grad, grad_cap);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void tp_seg_update(const int32_t* pos_s, const int32_t* segid, int64_t n, const int32_t* n_ent,
                   const float* psum, const int32_t* seg_start, const int32_t* n_uniq,
                   unsigned long long* acc, int64_t u_cap, const int64_t* slot_idx, void* slots,
                   int64_t cap, int algo, int lr_type, float alpha, float beta, float l1, float l2,
                   float grad_scale, float max_delta, double* stats, int acc_stripes,
                   uint32_t* hist, int nbins, int hist_stripes, double* metrics,
                   int64_t* step_counter, hipStream_t st) {
  if (n <= 0) return;
  if (hist && nbins != 2048) throw std::runtime_error("tp_seg_update: the fused AUC needs 2048 bins");
  const TpGeom g = tp_geom(n, 31);
  UpdateParams p{algo, lr_type, alpha, beta, l1, l2, grad_scale, max_delta};
  tp_seg_update_kernel<<<grid_for(g.N, 256, 2048), 256, 0, st>>>(
      pos_s, segid, g.N, n_ent, psum, g.N, seg_start, n_uniq, acc, u_cap, slot_idx,
      (Slot*)slots, cap, p, stats, acc_stripes, hist, nbins, hist_stripes, metrics, step_counter);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
