// Histogram tree engine for GBM / DRF / XGBoost / IsolationForest on MI355X (gfx950).
//
// Reference behaviour (what these kernels replace):
//   h2o-algos/src/main/java/hex/tree/ScoreBuildHistogram2.java  (per-chunk histogram accumulation)
//   h2o-algos/src/main/java/hex/tree/DHistogram.java            (w, wY, wYY bins + NA bin)
//   h2o-algos/src/main/java/hex/tree/DTree.java:984-1487         (findBestSplitPoint)
//   h2o-algos/src/main/java/hex/tree/gbm/GBM.java               (leaf Newton sums, prediction update)
//
// Design (MI355X-first, not a port):
//   * features are pre-binned once into a row-major uint8 matrix (bin 255 = NA), so a row is Fp bytes.
//   * rows are PHYSICALLY partitioned by tree node every level (stable two-pass partition: k_count ->
//     k_plan scan -> k_move_lean), so every histogram pass streams contiguous rows of ONE node and the
//     per-node histogram lives privately in LDS (fixed-point int64, see below).
//   * only the smaller child of each split is histogrammed (k_hist_build over its contiguous rows),
//     into a COMPACT buffer indexed by the parent (one built child per parent); the sibling comes
//     from parent - child (fused into k_hist_reduce, or into k_split_find on row-sharded levels), in fp64.
//     Row-sharded runs exchange only that compact buffer: half the bytes of every child slot of the level.
//   * split search, child planning, leaf numbering and tile planning all stay on device: a whole
//     tree is a fixed launch sequence with no host synchronisation.
//   * rows reaching a leaf write their leaf id in ORIGINAL row order (scatter through ridx) and stop
//     moving; the prediction update is then a coalesced elementwise op.
//   * wave64: 8 lanes own one row (one 32-bit word = 4 bins each), a wave covers 8 rows, so lanes of a
//     wave hit 8 different feature sub-histograms (few same-address LDS atomic collisions).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "abi.h"

#define NBIN 256
#define AMAX_SHARDS 64  // per-block |aux| maxima shards (k_amax / k_gbm_step -> k_qscale)
#define NA_BIN 255
#define FTILE 32                // features per LDS histogram tile
#define BLK 1024                // one 16-wave block per CU (the int64 LDS histogram is 128 KiB)
#define NW (BLK / 64)
#define TILE 2048               // rows per work tile
#define LEAFQ_STRIPES 16        // fixed-point leaf-sum copies (leafq: LEAFQ_STRIPES * 2 * leaf_cap slots)
#define LPR 8                   // lanes per row
#define RPI (BLK / LPR)         // rows per iteration (128)

struct Node {      // one active node of a level (rows [start, start+len) of the level's buffer)
  int start, len, build, parent, sib /*other active child of the parent, or -1*/,
      dir /*odd levels: 0 left / 1 right child*/, pad1, pad2;
};

#define NBW 32     // 32-bit words of a decision bitset: 1024 bins (the levels of a wide-categorical group)
#define GROUP_CAT 2
struct Dec {       // split decision (176 B)
  int feat;        // -1: no split (terminal)
  int bin;         // numeric: data bins < bin go left; group split: the group's packed 'elsewhere' bytes
  int na_left;     // NA rows go left?
  int is_cat;      // categorical: bitset `bits` over bins -> 1 = left; GROUP_CAT: a wide-categorical group
                   // (columns feat..feat+3, one aligned row word; bits over the global bins 254k + b)
  unsigned bits[NBW];
  double gain;     // improvement (for variable importance)
  double wl, wr;   // weighted row counts left/right
  float predl, predr;
};

#define TP_MAXL_DEV 64   // deepest tree the native plan walks (TreePlan arrays hold TP_MAXL = 65 levels)

struct Cand {      // best split of one (node, feature)
  double expl;     // explained "variance" of the split (larger is better)
  double gain;
  double wl, wr;
  float predl, predr;
  int bin, na_left, valid, is_cat;
  unsigned bits[NBW];
};

struct SplitParams {
  double min_w;            // min_rows (SE mode) / min_child_weight (Newton mode)
  double min_split_improvement;
  double lambda, alpha, gamma;
  int mode;                // 0 = squared error (GBM/DRF, H2O semantics), 1 = Newton (XGBoost), 2 = random (IsoForest)
  int random_split;        // extremely randomized / isolation: pick a random threshold
  unsigned long long seed;
  int hist_type;           // numeric candidate lattice (with adapt_nb > 1): HT_* below
  int fcut;                // > 0: only columns < fcut are searched (narrow levels of wide numeric bins, TreePlan)
  // The reference's node range (DTree.java:337-375) for the adaptive lattices (range_on != 0): the root bins over
  // its columns' [min, max] (vrange: exact extremes of every column over ALL rows; the open-ended first / last bins
  // map to them); a node at depth >= 1 over the range its PARENT's histogram observed (hprev: the previous level's
  // node histograms, same slot layout), narrowed at the parent's numeric split (pdec) for every column of the split
  // feature (fgroup: engine column -> feature in bits 0-29; null = identity). Global column ids throughout (f + f0);
  // edges_all: [F][255] edges of every column (the split column's threshold value).
  const float* vrange;
  const double* hprev;
  const Dec* pdec;
  const Node* rnodes;
  const int* fgroup;
  const float* edges_all;
  int range_on, pad_r;
  // wide-categorical groups (Binning.gcat, null: none): a group's first column = its real columns (1..4), its
  // other columns -1; the first column's block searches one histogram over all of the group's levels
  const int* gcat;
};

// histogram types (SharedTreeParameters.HistogramType) as candidate lattices over the global bins
enum { HT_QUANTILES = 0, HT_UNIFORM = 1, HT_RANDOM = 2, HT_ROBUST = 3, HT_ROUND_ROBIN = 4 };

// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ bool dec_go_left(const Dec* d, int b) {
  // d points to global memory or LDS: the runtime-indexed bitset must not live in registers (scratch)
  if (b == NA_BIN) return d->na_left != 0;
  if (d->is_cat) return (d->bits[b >> 5] >> (b & 31)) & 1u;
  return b < d->bin;
}

// the global bin (254k + byte) of a row of a wide-categorical group from its aligned group word: the one real
// column whose byte is not its 'elsewhere' bin (byte k of `pack`; 0 = padding) holds the level; -1 = NA
__device__ __forceinline__ int group_level(unsigned word, unsigned pack) {
  if ((word & 0xFFu) == NA_BIN) return -1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const unsigned ek = (pack >> (8 * k)) & 0xFFu, b = (word >> (8 * k)) & 0xFFu;
    if (ek != 0u && b != ek) return 254 * k + (int)b;
  }
  return -1;
}

// a decision on its row key: the split column's byte, or (GROUP_CAT) the group's aligned row word
template <bool GRP = true>
__device__ __forceinline__ bool dec_go_left_key(const Dec* d, unsigned v) {
  if (GRP && d->is_cat == GROUP_CAT) {
    const int l = group_level(v, (unsigned)d->bin);
    return l < 0 ? d->na_left != 0 : ((d->bits[l >> 5] >> (l & 31)) & 1u) != 0u;
  }
  return dec_go_left(d, (int)v);
}

// node index of tile t: largest i with tile_prefix[i] <= t
__device__ __forceinline__ int find_node(const int* __restrict__ tp, int n, int t) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (tp[mid] <= t) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ double wave_sum_d(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-reduce 4 doubles (BLK threads), result valid in thread 0.
__device__ void block_sum4(double v[4], double* scratch /* >= 4*(BLK/64) */) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int k = 0; k < 4; ++k) v[k] = wave_sum_d(v[k]);
  __syncthreads();
  if (lane == 0) for (int k = 0; k < 4; ++k) scratch[k * 16 + wid] = v[k];
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 0; k < 4; ++k) { double s = 0; for (int w = 0; w < nw; ++w) s += scratch[k * 16 + w]; v[k] = s; }
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// LDS histogram. MEASURED on gfx950 (scripts/mb_lds_atomic.hip): ds_add_f32 runs ~12x slower than
// integer LDS atomics (3.04 ms vs 0.25 ms for 11M x 28 updates), so bins accumulate in FIXED POINT:
// every row's (w, wY) is scaled by a per-tree 2^40/max|.| and added as int64 (ds_add_u64). The sums
// are exact and order independent (deterministic histograms); flushes convert to fp64 globally.
//
// Layout (int64), BANK-CONFLICT FREE for the atomics: entry (feature fl, bin) of plane r (0: w or packed,
// 1: wY) sits at r * HPLANE + bin * FTILE + fslot(fl). A ds_add_u64 wave-instruction is served in four
// 16-lane groups (2 rows x 8 words, bank = dword address mod 32); each lane adds feature 4*word + k of its
// row, with k rotated by the row's parity (hist_rows), and fslot() places features 4j+k and 4(j+4)+k two
// bank pairs apart, so the 16 lanes of a group always hit 16 distinct bank pairs whatever the bins are.
// (The former [feature][bin] layout put random bins on random banks: 3-4 way conflicts per group.)
// Plane 1 is offset by 16 entries so the flush's (r = 0, 1) lane pairs read disjoint banks.
// nayy (fp32 NA-bin wYY, rare) follows the planes.
#define HPLANE (NBIN * FTILE + 16)
#define HIST_LDS_BYTES (2 * HPLANE * 8 + FTILE * 4)
#define WQCAP 192   // FILT: per-wave queue of selected rows (< 64 carried over + one tile's 128 rows)
#define HIST_LDS_TAIL (64 * 8 + (BLK / 64) * WQCAP * 4)   // red + FILT per-wave row queues
__device__ __forceinline__ int fslot(int fl) { return (fl & 16) | ((fl + ((fl >> 4) << 1)) & 15); }

__device__ __forceinline__ void lds_zero64(long long* h, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) h[i] = 0ll;
}

__device__ __forceinline__ long long q64(float v, float scale) {
  return (long long)(v * scale);   // |v*scale| <= 2^40: exact conversion of the fp32 product
}

// PACKED mode (row weights are 0 / 1: unit weights or a sample mask): ONE ds_add_u64 per (row, feature) instead of
// two — count in bits [48, 64) as an UNSIGNED 16-bit field, wY in the low 48 bits as signed fixed point scaled to
// |q| <= 2^30 per row (one v_cvt_i32_f32 per row). A flush window holds < 2^16 rows (PACK_MAX), so the signed low part
// stays inside +-2^46 and the count never carries out: decode with one logical shift of the biased value.
// (r5: the window was 15 tiles with a signed count field, so a root block of 11M / 256 = 43K rows flushed twice, the
// second flush reading its partial slot back; 31 tiles keep one flush per block at that size)
#define PACK_SHIFT 48
#define PACK_MAX 63488   // rows per LDS flush window in packed mode (31 tiles)
// FPACK (XGBoost: the row weight is a float hessian): the same one-atomic word with 32 / 32 fields, hessian
// * sw unsigned in the high half, wY * sp signed in the low half, both rounded to nearest; k_qscale sizes
// sw = 0.99 * 2^32 / (PACK_MAX * max h) and sp = 0.99 * 2^31 / (PACK_MAX * max |wY|), so a window never
// carries (~2^-15 of the largest row value per row: fp32-class histogram sums at half the LDS atomics).
// sw / shf come from qs[10] / qs[12] (count mode: 1, 48); the branch is uniform over the kernel.
__device__ __forceinline__ long long qpack(float w, float b, float scale_p, float sw, float shf) {
  if (shf < 40.f) return ((long long)__float2uint_rn(w * sw) << 32) + (long long)__float2int_rn(b * scale_p);
  return ((long long)__float2int_rz(w) << PACK_SHIFT) + (long long)__float2int_rz(b * scale_p);
}
__device__ __forceinline__ void unpack(long long v, long long& cnt, long long& val, int shift = PACK_SHIFT) {
  cnt = (long long)(((unsigned long long)v + (1ull << (shift - 1))) >> shift);
  val = (long long)((unsigned long long)v - ((unsigned long long)cnt << shift));
}

// Flush of one block's LDS histogram into ITS OWN partial slot (plain stores, no global atomics):
// partial index = blockIdx.x + node (unique: a block's tiles and nodes both increase, see k_hist_reduce).
// `acc` (a later packed flush window of the same node) adds into what this same thread stored before.
// Slot layout (bin-major): [256 bins][F][2] doubles, then [F] NA-wYY, then [1] node wYY. Lanes walk
// (bin, feature, r): consecutive global doubles and, in LDS, distinct fslot bank pairs per r plus the
// plane offset (conflict-free reads).
// MEASURED: the former fp64 atomicAdd flush into one shared slot cost ~30 us per level regardless of
// row count (256 blocks x 14K same-address atomics serialise in L2) — the fixed cost that dominated
// small shards (1.375M rows/GPU at 8 GPUs).
// f32: the slot holds floats (same slot stride): half the flush / reduce bytes; k_hist_reduce still sums in fp64
// in a fixed order. Exact per-block counts (< 2^24 rows per block) and ~6e-8 relative wY per partial.
template <typename P>
__device__ __forceinline__ void put_partial(P* q, double d, bool acc) {
  *q = acc ? (P)((double)*q + d) : (P)d;
}
// srep/snb (LDS, per tile feature): replica count and bin count of a low-cardinality feature whose updates were
// spread over `srep` copies of its bins (see hist_rows); bin b < nb is the sum of the copies b + c * nb.
__device__ void flush_partial(const long long* h, const float* nayy, double node_wyy, int ftile, int F,
                              double* __restrict__ part, const double* __restrict__ qs, bool packed, bool acc,
                              bool f32, const int* srep, const int* snb, const int* sfine) {
  const int f0 = ftile * FTILE;
  const int nf = min(FTILE, F - f0);
  const double inv_a = qs[2], inv_b = qs[3], inv_p = qs[5];
  if (packed) {
    const int pshift = (int)qs[12];
    const double inv_w = qs[11];
    // one packed u64 holds both planes of (bin, feature): a lane reads it once (replicas summed), unpacks once and
    // stores the (w, wY) pair with one 16-byte (8-byte f32) store
    const int dbin = (int)blockDim.x / nf, drem = (int)blockDim.x - dbin * nf;
    int bin = (int)threadIdx.x / nf, fl = (int)threadIdx.x - bin * nf;
    for (int i = threadIdx.x; i < nf * NBIN; i += blockDim.x, bin += dbin, fl += drem) {
      if (fl >= nf) { fl -= nf; ++bin; }
      const int reps = srep[fl], nb = snb[fl];
      long long q = 0;
      if (sfine[fl]) {
        const int m = fl & ~3, k = fl & 3;
#pragma unroll
        for (int l = 0; l < 4; ++l) {
          const int bb = l <= k ? bin : bin - 1;
          if (bb >= 0) q += h[bb * FTILE + fslot(m + l)];
        }
      } else if (reps == 1) {
        q = h[bin * FTILE + fslot(fl)];
      } else if (bin < nb) {
        for (int c = 0; c < reps; ++c) q += h[(bin + c * nb) * FTILE + fslot(fl)];
      }
      long long c, v;
      unpack(q, c, v, pshift);
      const double dc = (double)c * inv_w, dv = (double)v * inv_p;
      const size_t e2 = (size_t)bin * 2 * F + 2 * (f0 + fl);
      if (f32) {
        float2* p2 = (float2*)((float*)part + e2);
        float2 o = make_float2((float)dc, (float)dv);
        if (acc) { const float2 a = *p2; o = make_float2((float)((double)a.x + dc), (float)((double)a.y + dv)); }
        *p2 = o;
      } else {
        double2* p2 = (double2*)(part + e2);
        double2 o = make_double2(dc, dv);
        if (acc) { const double2 a = *p2; o.x += a.x; o.y += a.y; }
        *p2 = o;
      }
    }
  } else {
  // (bin, rem) of entry i advanced incrementally: no integer division per entry
  const int row2 = 2 * nf, dbin = (int)blockDim.x / row2, drem = (int)blockDim.x - dbin * row2;
  int bin = (int)threadIdx.x / row2, rem = (int)threadIdx.x - bin * row2;
  for (int i = threadIdx.x; i < nf * 2 * NBIN; i += blockDim.x, bin += dbin, rem += drem) {
    if (rem >= row2) { rem -= row2; ++bin; }
    const int fl = rem >> 1, r = rem & 1;
    const int reps = srep[fl], nb = snb[fl];
    long long q = 0;                       // the entry's fixed-point value (plane r), replicas summed
    if (sfine[fl]) {
      // column k of a fine group: bin b holds fine bins t = 4h + l with h + [l > k] == b, i.e. entries
      // (b, l <= k) and (b - 1, l > k) of the fine histogram (NA: t = 1020 = entry (255, 0))
      const int m = fl & ~3, k = fl & 3;
      const int pl = r * HPLANE;
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        const int bb = l <= k ? bin : bin - 1;
        if (bb >= 0) q += h[pl + bb * FTILE + fslot(m + l)];
      }
    } else if (reps == 1 || bin < nb) {
      for (int c = 0; c < reps; ++c) q += h[r * HPLANE + (bin + c * nb) * FTILE + fslot(fl)];
    }
    const double d = (double)q * (r ? inv_b : inv_a);
    const size_t e2 = (size_t)bin * 2 * F + 2 * (f0 + fl) + r;
    if (f32) put_partial((float*)part + e2, d, acc);
    else put_partial(part + e2, d, acc);
  }
  }
  for (int i = threadIdx.x; i < nf; i += blockDim.x) {
    const size_t e2 = (size_t)F * 2 * NBIN + f0 + i;
    if (f32) put_partial((float*)part + e2, (double)nayy[i], acc);
    else put_partial(part + e2, (double)nayy[i], acc);
  }
  if (threadIdx.x == 0 && ftile == 0) {
    const size_t e2 = (size_t)F * 2 * NBIN + F;
    if (f32) put_partial((float*)part + e2, node_wyy, acc);
    else put_partial(part + e2, node_wyy, acc);
  }
}

__device__ __forceinline__ float row_yy(float a, float b) {
  return a > 0.f ? b * b * __builtin_amdgcn_rcpf(a) : 0.f;
}

// Parent-decision filter of an odd-level histogram (k_hist_build<true>): only rows of the parent's
// range that go to `dir` are accumulated; `count` lanes tally the parent's left-goers. The numeric
// test runs on registers; only categorical splits read the bitset (LDS copy of the decision).
// Bins layouts. Row-major: row r's F feature bytes at r * stride. PLANAR (F > 32): 32-feature planes,
// feature f of row r at ((f >> 5) * N + r) * 32 + (f & 31) — the histogram block of feature tile t reads
// only plane t (32 B per row) instead of pulling every 64-B row line once per feature tile.
__device__ __forceinline__ size_t bin_off(long long row, int f, int stride, long long N, int planar) {
  return planar ? ((size_t)(f >> 5) * (size_t)N + (size_t)row) * 32 + (f & 31) : (size_t)row * stride + f;
}

struct RowFilter {
  const Dec* pd;   // parent decision (LDS copy)
  const uint8_t* fptr;   // byte of the split feature in row 0 (layout-aware); row r at fptr[r * fstride]
  int fstride;
  int feat;        // its split feature
  int jw;          // lane (within the 8-lane row group) whose word holds `feat`, or -1: load the byte
  int dir;         // 0: accumulate left-goers, 1: right-goers
  int bin, na_left, is_cat;
  bool count;
  __device__ __forceinline__ bool left(unsigned v) const {
    if (is_cat == GROUP_CAT) {              // v: the group's aligned row word
      const int l = group_level(v, (unsigned)bin);
      return l < 0 ? na_left != 0 : ((pd->bits[l >> 5] >> (l & 31)) & 1u) != 0u;
    }
    const int b = (int)v;
    if (b == NA_BIN) return na_left != 0;
    if (is_cat) return (pd->bits[b >> 5] >> (b & 31)) & 1u;
    return b < bin;
  }
};


// Histogram rows [r0, r1) of one node into LDS: lane group g (8 lanes, one 4-feature row word each)
// takes rows g, g + RPI, ...; UNR rows per lane group are loaded before any atomic.
// MEASURED: this loop is VALU-issue bound, not memory bound (prefetching / 4..16 rows in flight all ran
// within 1.5 %), so everything per-lane is hoisted: the 4 feature slots and byte shifts of the lane's word
// (rotated by row parity, see the layout note), feature validity, and an all-bytes NA test per word; the
// common row is then bfe + lshl_add + ds_add_u64 per feature (two atomics when not PACKED).
// FILT (odd levels): the rows of a parent tile that the parent's decision sends to the built child, as an
// ascending row list in LDS (one lane per row tests the split byte; wave ballots + a (pass, wave) prefix
// place them). The histogram loop then runs over full lane groups of selected rows: filtering inside it
// left about half of each wave's lanes idle through the atomics (the loop is issue-bound), so a filtered
// pass cost two plain passes. ftile-0 blocks also count the parent's left-goers (nl_out).
// orders LDS accesses of different lanes of one wave (compiler and hardware), without a block barrier
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#define FNP (TILE / BLK)   // FILT: rows per lane of a tile
#define WROWS (TILE / NW)   // FILT: rows of a tile per wave (a contiguous 128-row slice)
// split-feature bytes of this lane's rows of its wave's slice of tile [r0, r1) (rows past r1 load row r1 - 1,
// unused)
__device__ __forceinline__ void filt_load(const RowFilter& flt, int r0, int r1, unsigned (&byt)[FNP]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (flt.is_cat == GROUP_CAT) {          // a wide-categorical group split: the group's aligned row word
#pragma unroll
    for (int p = 0; p < FNP; ++p) {
      const int row = min(r0 + wv * WROWS + p * 64 + lane, r1 - 1);
      byt[p] = *reinterpret_cast<const unsigned*>(flt.fptr + (size_t)row * (size_t)flt.fstride);
    }
    return;
  }
#pragma unroll
  for (int p = 0; p < FNP; ++p) {
    const int row = min(r0 + wv * WROWS + p * 64 + lane, r1 - 1);
    byt[p] = flt.fptr[(size_t)row * (size_t)flt.fstride];
  }
}

// WAVE-LOCAL compaction (no block barrier): the wave appends the rows of its tile slice that the parent's
// decision sends to the built child to its own LDS queue wq (ascending), after the qn rows still queued.
// MEASURED before (block-wide list, two __syncthreads per tile): every wave waited on the slowest wave's
// split-byte loads and then on the gathers, with nothing to overlap them — the filtered pass over half the
// rows cost as much as a plain pass over all of them.
__device__ __forceinline__ int filt_append(const RowFilter& flt, int r0, int r1, int* wq, int qn, int& lcnt,
                                           const unsigned (&byt)[FNP]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int p = 0; p < FNP; ++p) {
    const int row = r0 + wv * WROWS + p * 64 + lane;
    bool sl = false;
    if (row < r1) {
      const bool gl = flt.left(byt[p]);
      if (flt.count) lcnt += gl ? 1 : 0;
      sl = (gl ? 0 : 1) == flt.dir;
    }
    const unsigned long long m = __ballot(sl);
    if (sl) wq[qn + __popcll(m & below)] = row;
    qn += __popcll(m);
  }
  return qn;
}

#ifndef H2O_UNR
#define H2O_UNR 8
#endif
// hist: rows per lane group loaded before any atomic (UNR independent loads per lane; the FILT queue batches use 8)

// Row loads of the histogram loop. BUF: 32-bit buffer offsets into the bins (rows of 2^lgw bytes) and the aux planes
// (each < 4 GiB; the host checks): one shift per row and per-unroll SGPR offsets instead of a 64-bit multiply-add
// per load (the loop is VALU-issue bound, see hist_rows).
struct HistSrc {
  const unsigned* bins32;
  const float* aw;
  const float* ay;
  __amdgpu_buffer_rsrc_t rb, ra, rw;
  int lgw;
};

__device__ __forceinline__ HistSrc make_src(const unsigned* bins32, const float* aw, const float* ay, long long N, int W,
                                            int lgw) {
  // (descriptors are built unconditionally: a few SALU; only BUF kernels use them)
  return HistSrc{bins32, aw, ay,
                 __builtin_amdgcn_make_buffer_rsrc((void*)bins32, 0, (int)(unsigned)((unsigned long long)N * W * 4),
                                                   0x00020000),
                 __builtin_amdgcn_make_buffer_rsrc((void*)ay, 0, (int)(unsigned)(N * 4), 0x00020000),
                 __builtin_amdgcn_make_buffer_rsrc((void*)(aw ? aw : ay), 0, (int)(unsigned)(N * 4), 0x00020000),
                 lgw};
}

// MEASURED (r4, 11M x 28 HIGGS shape, same-box A/B): the plain pass issues 11M x 28 = 308M ds_add_u64 in ~131 us,
// one wave-level atomic per ~16 cycles per CU: it runs at the LDS atomic rate. Software-pipelining the row batches
// across merged same-node tiles changed nothing (1.376-1.394 vs 1.380-1.388 ms/tree), a 64-VGPR build with two
// blocks per CU was 13 % slower (spills), 512 / 384 blocks per launch 5-8 % slower (more partials), and spreading
// low-cardinality features over bin replicas removed the SQ_LDS_ADDR_CONFLICT cycles (1.8e8 -> 5e6) at equal time.
// Histogram rows [r0, r1) of one node into LDS (FILT: entries [r0, r1) of the LDS row list): lane group g
// (8 lanes, one 4-feature row word each) takes rows g, g + GR, ...; UNR rows per lane group are loaded
// before any atomic.
// MEASURED: this loop is VALU-issue bound, not memory bound (prefetching / 4..16 rows in flight all ran
// within 1.5 %), so everything per-lane is hoisted: the 4 feature slots and byte shifts of the lane's word
// (rotated by row parity, see the layout note), feature validity; NONA (no NA bin anywhere, a launch-time
// property of the bins) drops the per-word NA test at compile time; a batch wholly inside the node skips the
// per-row bounds tests; BUF addresses with 32-bit offsets. The common row is then bfe + lshl_add + ds_add_u64
// per feature (two atomics when not PACKED).
template <bool FILT, bool PACKED, bool UNIT, bool NONA, bool BUF, bool FINE, int GR = RPI, int UNR = H2O_UNR>
__device__ __forceinline__ void hist_rows(long long* h, float* nayy, const HistSrc& src, int W, int wabs,
                                          int F, bool lead, int r0, int r1, int g, int j, float& wyy, float sa,
                                          float sb, float sp, const int* lst, const int* srep, const int* snb,
                                          const int* sfine) {
  const int rot = g & 1;
  unsigned offb[4], sh[4];           // byte offset of the lane's feature slot in a bin row; its byte's shift
  unsigned vmask = 0u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int kk = (k + rot) & 3;
    const int fl = j * 4 + kk;
    // low-cardinality features (srep > 1, NONA only): same-parity rows of a lane group collide on the few bins of
    // such a feature (SQ_LDS_ADDR_CONFLICT ~ SQ_LDS_IDX_ACTIVE on HIGGS-like data with 3-valued b-tags); their
    // updates go to copy (g >> 1) mod srep of the feature's bins, summed by the flush
    const int c = (g >> 1) & (srep[fl] - 1);
    offb[k] = (unsigned)fslot(fl) * 8u + ((unsigned)(c * snb[fl]) << 8);
    sh[k] = 8u * kk;
    if (wabs < W && wabs * 4 + kk < F) vmask |= 0xFFu << (8 * kk);
  }
  const bool live = vmask != 0u;     // a lane whose word is past the row adds nothing (no dummy atomics)
  // FINE word: the 4 bytes are the 4 interleaved engine columns of ONE wide numeric feature (ops/binning.py), so
  // their byte sum is the fine bin t = #{edges <= x} (NA: 4 x 255 = 1020) and one atomic into fine entry
  // (bin t >> 2, column t & 3) replaces four; the flush rebuilds the four column histograms from the fine one
  const bool fine = FINE && live && sfine[j * 4] != 0;
  unsigned fsl[4];
#pragma unroll
  for (int l = 0; l < 4; ++l) fsl[l] = (unsigned)fslot(j * 4 + l) * 8u;
  const int wc = min(wabs, W - 1);
  const bool weighted = !UNIT && src.aw != nullptr;
  char* Hb = (char*)h;
  // entry (bin, slot) at byte (bin * FTILE + slot) * 8 = (bin << 8) + offb: one v_bfe_u32 + one v_lshl_add_u32
  // per atomic (MEASURED: the shift / and / shift / add form the compiler made of the index expression was 4 VALU
  // per atomic, and this loop is VALU-issue bound: ~12 VALU per LDS instruction in rocprofv3 PMC)
  static_assert(FTILE * 8 == 256, "bin row of the LDS histogram is 256 bytes");
  auto ent = [&](unsigned w, int k) -> unsigned long long* {
    return (unsigned long long*)(Hb + ((__builtin_amdgcn_ubfe(w, sh[k], 8) << 8) + offb[k]));
  };
  for (int base = r0; base < r1; base += GR * UNR) {
    unsigned wd[UNR];
    float2 ab[UNR];
    const bool whole = base + GR * UNR <= r1;          // block-uniform: no row of the batch is past r1
    if (BUF && !FILT && whole) {
      // consecutive rows: one voffset per batch, the unroll steps are SGPR offsets
      const unsigned row0 = (unsigned)(base + g);
      const unsigned vb = (row0 << src.lgw) + (unsigned)wc * 4u, va = row0 * 4u;
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        wd[u] = __builtin_amdgcn_raw_buffer_load_b32(src.rb, vb, (unsigned)(u * GR) << src.lgw, 0);
        const float y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(src.ra, va, u * GR * 4, 0));
        const float w = weighted ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(src.rw, va, u * GR * 4, 0))
                                 : 1.f;
        ab[u] = make_float2(w, y);
      }
    } else {
      // unconditional loads (rows clamped into the node, words into the row): no exec-mask branches here;
      // rows past r1 are skipped below, invalid words have vmask == 0
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int idx = whole ? base + g + u * GR : min(base + g + u * GR, r1 - 1);
        const int row = FILT ? lst[idx] : idx;
        if (BUF) {
          const unsigned ro = (unsigned)row;
          wd[u] = __builtin_amdgcn_raw_buffer_load_b32(src.rb, (ro << src.lgw) + (unsigned)wc * 4u, 0, 0);
          const float y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(src.ra, ro * 4u, 0, 0));
          const float w = weighted ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(src.rw, ro * 4u, 0, 0)) : 1.f;
          ab[u] = make_float2(w, y);
        } else {
          // SoA aux planes: wY always, w only when rows are weighted (aw == null: unit weights)
          ab[u] = make_float2(weighted ? src.aw[row] : 1.f, src.ay[row]);
          wd[u] = src.bins32[(size_t)row * W + wc];
        }
      }
    }
    // One row word: every live lane adds all 4 of its word's features, valid or not: a feature past F (a partial last
    // word) has the slot of a feature >= the tile's count, an LDS column the flush never reads, so its atomics are
    // harmless — no divergent full / partial paths (the former per-row exec-mask juggling cost ~10 SALU per row).
    // Only the rare NA-bin yy tally branches.
    auto row = [&](int u) {
      // UNIT (packed, every row weight exactly 1): constant count part, yy = wY^2 (no reciprocal)
      if (lead) wyy += UNIT ? ab[u].y * ab[u].y : row_yy(ab[u].x, ab[u].y);
      // (int) conversion truncates toward zero (v_cvt_i32_f32): the __float2int_rz form added a v_trunc_f32
      const long long qa = UNIT ? (1ll << PACK_SHIFT) + (long long)(int)(ab[u].y * sp)
                                : PACKED ? qpack(ab[u].x, ab[u].y, sp, sa, sb) : q64(ab[u].x, sa);
      const long long qb = PACKED ? 0ll : q64(ab[u].y, sb);
      const unsigned w = wd[u];
      if (FINE && fine) {
        const unsigned t = __builtin_amdgcn_sad_u8(w, 0u, 0u);          // sum of the 4 bytes
        const unsigned l = t & 3u;
        const unsigned so = (l & 2u) ? ((l & 1u) ? fsl[3] : fsl[2]) : ((l & 1u) ? fsl[1] : fsl[0]);
        unsigned long long* p = (unsigned long long*)(Hb + (((t >> 2) << 8) + so));
        atomicAdd(p, (unsigned long long)qa);
        if (!PACKED) atomicAdd(p + HPLANE, (unsigned long long)qb);
      } else if (live) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          unsigned long long* p = ent(w, k);
          atomicAdd(p, (unsigned long long)qa);
          if (!PACKED) atomicAdd(p + HPLANE, (unsigned long long)qb);
        }
      }
      if (!NONA) {
        const unsigned x = ~w | ~vmask;                   // a zero byte of x = an NA bin of a valid feature
        if (((x - 0x01010101u) & ~x & 0x80808080u) != 0u) {
          const float yy = UNIT ? ab[u].y * ab[u].y : row_yy(ab[u].x, ab[u].y);
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (((vmask >> sh[k]) & 1u) && __builtin_amdgcn_ubfe(w, sh[k], 8) == NA_BIN)
              atomicAdd(nayy + j * 4 + (sh[k] >> 3), yy);
        }
      }
    };
    if (whole) {
#pragma unroll
      for (int u = 0; u < UNR; ++u) row(u);
    } else {
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (base + g + u * GR < r1) row(u);
    }
  }
}

// Plain (non-FILT) histogram of node rows [r0, r1) — one contiguous run of a node inside the block's tile range (a
// whole window, not a tile): the per-lane setup runs once per run, and the loads of batch k + 1 are issued before the
// atomics of batch k (double-buffered registers), so the wave's next rows are in flight while it feeds the LDS.
// MEASURED (r5, scripts/mb_hist4.hip, 11M x 28): the pure LDS atomic rate is 8 cycles per ds_add_u64 wave-instruction
// per CU (63 us for 308M updates) and the loads alone stream at ~6 TB/s (68 us); the per-tile loop with a per-row
// fine / live branch reached only 135 us.
template <bool PACKED, bool UNIT, bool NONA, bool BUF, bool FINE>
__device__ __forceinline__ void hist_span(long long* h, float* nayy, const HistSrc& src, int W, int wabs, int F,
                                          bool lead, int r0, int r1, int g, int j, float& wyy, float sa, float sb,
                                          float sp, const int* srep, const int* snb, const int* sfine,
                                          bool no_atoms = false) {
  constexpr int GR = RPI, UNR = H2O_UNR;
  const int rot = g & 1;
  unsigned offb[4], sh[4];
  unsigned vmask = 0u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int kk = (k + rot) & 3;
    const int fl = j * 4 + kk;
    const int c = (g >> 1) & (srep[fl] - 1);
    offb[k] = (unsigned)fslot(fl) * 8u + ((unsigned)(c * snb[fl]) << 8);
    sh[k] = 8u * kk;
    if (wabs < W && wabs * 4 + kk < F) vmask |= 0xFFu << (8 * kk);
  }
  const bool live = vmask != 0u && !no_atoms;
  const bool fine = FINE && live && sfine[j * 4] != 0;
  unsigned fsl[4];
#pragma unroll
  for (int l = 0; l < 4; ++l) fsl[l] = (unsigned)fslot(j * 4 + l) * 8u;
  const int wc = min(wabs, W - 1);
  const bool weighted = !UNIT && src.aw != nullptr;
  char* Hb = (char*)h;
  auto load = [&](int base, unsigned (&wd)[UNR], float2 (&ab)[UNR]) {
    if (BUF && base + GR * UNR <= r1) {
      const unsigned row0 = (unsigned)(base + g);
      const unsigned vb = (row0 << src.lgw) + (unsigned)wc * 4u, va = row0 * 4u;
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        wd[u] = __builtin_amdgcn_raw_buffer_load_b32(src.rb, vb, (unsigned)(u * GR) << src.lgw, 0);
        const float y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(src.ra, va, u * GR * 4, 0));
        const float w = weighted ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(src.rw, va, u * GR * 4, 0))
                                 : 1.f;
        ab[u] = make_float2(w, y);
      }
    } else {
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int row = min(base + g + u * GR, r1 - 1);
        if (BUF) {
          const unsigned ro = (unsigned)row;
          wd[u] = __builtin_amdgcn_raw_buffer_load_b32(src.rb, (ro << src.lgw) + (unsigned)wc * 4u, 0, 0);
          const float y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(src.ra, ro * 4u, 0, 0));
          const float w = weighted ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(src.rw, ro * 4u, 0, 0)) : 1.f;
          ab[u] = make_float2(w, y);
        } else {
          ab[u] = make_float2(weighted ? src.aw[row] : 1.f, src.ay[row]);
          wd[u] = src.bins32[(size_t)row * W + wc];
        }
      }
    }
  };
  unsigned wdn[UNR];
  float2 abn[UNR];
  if (r0 < r1) load(r0, wdn, abn);
  for (int base = r0; base < r1; base += GR * UNR) {
    unsigned wd[UNR];
    float2 ab[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) { wd[u] = wdn[u]; ab[u] = abn[u]; }
    if (base + GR * UNR < r1) load(base + GR * UNR, wdn, abn);
    auto atoms = [&](int u) {
      const long long qa = UNIT ? (1ll << PACK_SHIFT) + (long long)(int)(ab[u].y * sp)
                                : PACKED ? qpack(ab[u].x, ab[u].y, sp, sa, sb) : q64(ab[u].x, sa);
      const long long qb = PACKED ? 0ll : q64(ab[u].y, sb);
      const unsigned w = wd[u];
      if (FINE && fine) {
        const unsigned t = __builtin_amdgcn_sad_u8(w, 0u, 0u);
        const unsigned l = t & 3u;
        const unsigned so = (l & 2u) ? ((l & 1u) ? fsl[3] : fsl[2]) : ((l & 1u) ? fsl[1] : fsl[0]);
        unsigned long long* p = (unsigned long long*)(Hb + (((t >> 2) << 8) + so));
        atomicAdd(p, (unsigned long long)qa);
        if (!PACKED) atomicAdd(p + HPLANE, (unsigned long long)qb);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          unsigned long long* p = (unsigned long long*)(Hb + ((__builtin_amdgcn_ubfe(w, sh[k], 8) << 8) + offb[k]));
          atomicAdd(p, (unsigned long long)qa);
          if (!PACKED) atomicAdd(p + HPLANE, (unsigned long long)qb);
        }
      }
    };
    auto row = [&](int u) {
      if (lead) wyy += UNIT ? ab[u].y * ab[u].y : row_yy(ab[u].x, ab[u].y);
      if (FINE && live) atoms(u);
      if (!NONA) {
        const unsigned w = wd[u];
        const unsigned x = ~w | ~vmask;
        if (((x - 0x01010101u) & ~x & 0x80808080u) != 0u) {
          const float yy = UNIT ? ab[u].y * ab[u].y : row_yy(ab[u].x, ab[u].y);
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (((vmask >> sh[k]) & 1u) && __builtin_amdgcn_ubfe(w, sh[k], 8) == NA_BIN)
              atomicAdd(nayy + j * 4 + (sh[k] >> 3), yy);
        }
      }
    };
    // !FINE: the lane's live test (a lane whose word holds no feature of the tile issues no atomics) is ONE exec-mask
    // branch around the batch's atomics, not one per row
    if (base + GR * UNR <= r1) {
#pragma unroll
      for (int u = 0; u < UNR; ++u) row(u);
      if (!FINE && live) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) atoms(u);
      }
    } else {
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (base + g + u * GR < r1) row(u);
      if (!FINE && live) {
#pragma unroll
        for (int u = 0; u < UNR; ++u)
          if (base + g + u * GR < r1) atoms(u);
      }
    }
  }
}

// FILT (odd levels), software-pipelined: a wave gathers the rows of its NEXT 64-row queue batch (one row per 8-lane
// group and step, UNR = 8 steps) and only then issues the atomics of the batch gathered before, so the gathers' latency
// hides behind that batch's atomics. MEASURED (r5 PMC, 11M HIGGS): the unpipelined filtered pass spent 55 % of its
// wave cycles waiting on memory (SQ_WAIT_ANY), each batch's gathers exposed in full.
struct FiltLane {   // per-lane setup of a FILT kernel (constant per block: feature tile and lane group fixed)
  unsigned offb[4];  // byte offset of the slot of byte k of the ROTATED word (see filt_atoms)
  unsigned vmask;    // valid features of the lane's word, in the original byte order
  int wc, rot;
  bool live, fine, weighted, lead;
};

template <bool PACKED, bool UNIT, bool FINE>
__device__ __forceinline__ FiltLane filt_lane(const HistSrc& src, int W, int wabs, int F, int g8, int j, bool lead,
                                              const int* srep, const int* snb, const int* sfine) {
  FiltLane L;
  L.rot = g8 & 1;
  L.vmask = 0u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int kk = (k + L.rot) & 3;
    const int fl = j * 4 + kk;
    const int c = (g8 >> 1) & (srep[fl] - 1);
    L.offb[k] = (unsigned)fslot(fl) * 8u + ((unsigned)(c * snb[fl]) << 8);
    if (wabs < W && wabs * 4 + kk < F) L.vmask |= 0xFFu << (8 * kk);
  }
  L.live = L.vmask != 0u;
  L.fine = FINE && L.live && sfine[j * 4] != 0;
  L.wc = min(wabs, W - 1);
  L.weighted = !UNIT && src.aw != nullptr;
  L.lead = lead;
  return L;
}

// gather the queued rows wq[0, n) (entry g8 + 8u per step; entries past n load row wq[n - 1], unused)
template <bool UNIT, bool BUF>
__device__ __forceinline__ void filt_gather(const FiltLane& L, const HistSrc& src, int W, const int* wq, int n, int g8,
                                            unsigned (&wd)[8], float (&yv)[8], float (&wv)[8]) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int row = wq[min(g8 + 8 * u, n - 1)];
    if (BUF) {
      const unsigned ro = (unsigned)row;
      wd[u] = __builtin_amdgcn_raw_buffer_load_b32(src.rb, (ro << src.lgw) + (unsigned)L.wc * 4u, 0, 0);
      yv[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(src.ra, ro * 4u, 0, 0));
      if (!UNIT) wv[u] = L.weighted ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(src.rw, ro * 4u, 0, 0)) : 1.f;
    } else {
      yv[u] = src.ay[row];
      if (!UNIT) wv[u] = L.weighted ? src.aw[row] : 1.f;
      wd[u] = src.bins32[(size_t)row * W + L.wc];
    }
  }
}

// the atomics (and NA / yy tallies) of a gathered batch of n rows. The word is rotated by the lane group's parity
// (byte k of the rotated word = feature 4j + ((k + rot) & 3), one v_alignbyte per row) so the byte extracts use
// constant shifts; same-parity rows of a 16-lane group then add distinct features (bank-conflict-free layout).
template <bool PACKED, bool UNIT, bool NONA, bool FINE>
__device__ __forceinline__ void filt_atoms(const FiltLane& L, long long* h, float* nayy, int n, int g8, int j,
                                           const unsigned (&wd)[8], const float (&yv)[8], const float (&wv)[8],
                                           float& wyy, float sa, float sb, float sp) {
  char* Hb = (char*)h;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    if (g8 + 8 * u >= n) continue;
    const float x = UNIT ? 1.f : wv[u];
    if (L.lead) wyy += UNIT ? yv[u] * yv[u] : row_yy(x, yv[u]);
    const long long qa = UNIT ? (1ll << PACK_SHIFT) + (long long)(int)(yv[u] * sp)
                              : PACKED ? qpack(x, yv[u], sp, sa, sb) : q64(x, sa);
    const long long qb = PACKED ? 0ll : q64(yv[u], sb);
    const unsigned w = wd[u];
    if (FINE && L.fine) {
      const unsigned t = __builtin_amdgcn_sad_u8(w, 0u, 0u);
      const unsigned l = t & 3u;
      unsigned long long* p = (unsigned long long*)(Hb + (((t >> 2) << 8) + (unsigned)fslot(j * 4 + (int)l) * 8u));
      atomicAdd(p, (unsigned long long)qa);
      if (!PACKED) atomicAdd(p + HPLANE, (unsigned long long)qb);
    } else if (L.live) {
      const unsigned wr = __builtin_amdgcn_alignbyte(w, w, L.rot);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        unsigned long long* p = (unsigned long long*)(Hb + ((__builtin_amdgcn_ubfe(wr, 8 * k, 8) << 8) + L.offb[k]));
        atomicAdd(p, (unsigned long long)qa);
        if (!PACKED) atomicAdd(p + HPLANE, (unsigned long long)qb);
      }
    }
    if (!NONA) {
      const unsigned xx = ~w | ~L.vmask;
      if (((xx - 0x01010101u) & ~xx & 0x80808080u) != 0u) {
        const float yy = UNIT ? yv[u] * yv[u] : row_yy(x, yv[u]);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (((L.vmask >> (8 * k)) & 1u) && __builtin_amdgcn_ubfe(w, 8 * k, 8) == NA_BIN) atomicAdd(nayy + j * 4 + k, yy);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// k_hist_build: histograms of all nodes with build==1 of a level, as per-block PARTIAL slots
// (partials + (blockIdx.x + node) * slot_doubles); k_hist_reduce sums them per node in a fixed order
// (deterministic, no global atomics). grid = (G, n_ftiles); each block takes a contiguous tile range.
// FILT (odd levels): a node's tiles cover its PARENT's rows; only rows the parent's decision sends to
// this child are accumulated, and ftile-0 blocks add the parent's left-going row count to nl_out.
template <bool FILT, bool PACKED, bool UNIT, bool NONA, bool BUF, bool FINE>
__global__ __launch_bounds__(BLK) void k_hist_build(
    const uint8_t* __restrict__ bins, int stride /*bytes per row, multiple of 4*/,
    const float* __restrict__ aw /*row weights or null (unit)*/, const float* __restrict__ ay /*w * Y*/,
    const Node* __restrict__ nodes, const int* __restrict__ tile_prefix,
    const int* __restrict__ meta /*[0]=n_nodes [2]=n_build_tiles*/, int F, double* __restrict__ partials,
    int slot_doubles, const double* __restrict__ qs /*[sa, sb, 1/sa, 1/sb, sp, 1/sp]*/,
    const Dec* __restrict__ pdec, int* __restrict__ nl_out, int f32, long long N, int planar, int lgw,
    const int* __restrict__ nbins_f /*[F] (NONA: low-cardinality spreading) or null*/,
    const int* __restrict__ fine_f /*[F] 1 = column of an aligned 4-column wide numeric group, or null*/,
    const uint8_t* __restrict__ fdir /*FILT: per row 0 = left / 1 = right of the parent split, or null*/,
    int dbg /*A/B diagnostics (H2O_HIST_DBG): bit 0 skips the partial flush, bit 1 the plain pass's atomics*/) {
  constexpr bool packed = PACKED;
  extern __shared__ __attribute__((aligned(16))) long long smem64[];
  long long* h = smem64;                                 // 2 planes (PACKED: 1 -> two blocks per CU fit)
  float* nayy = (float*)(smem64 + (PACKED ? 1 : 2) * HPLANE);   // FTILE
  double* red = (double*)(nayy + FTILE);                 // 64 doubles scratch
  const int lane = threadIdx.x & 63;
  int* wq = (int*)(red + 64) + (threadIdx.x >> 6) * WQCAP;   // FILT: this wave's queue of selected rows

  // tile_prefix here is the BUILD-tile prefix (only nodes with build=1 own tiles) and meta[2] the number
  // of build tiles: blocks split only the rows that are histogrammed (no idle blocks on skipped siblings)
  const int n_nodes = meta[0], n_tiles = meta[2];
  if (n_nodes <= 0 || n_tiles <= 0) return;
  const int per = (n_tiles + gridDim.x - 1) / gridDim.x;
  const int t0 = blockIdx.x * per, t1 = min(n_tiles, t0 + per);
  if (t0 >= t1) return;
  // (MEASURED: an XCD-aware 1-D order putting the feature-tile blocks of one row range on the same XCD
  // made XGBoost 100M x 50 histograms 9-20 % SLOWER — 4.56 -> 4.97 ms filtered, 2.32 -> 2.80 ms plain)
  const int ftile = blockIdx.y;
  planar &= 1;
  // planar: this block reads only its 32-feature plane (8 words per row, features counted from the plane)
  const int W = planar ? LPR : stride >> 2;
  const int g = threadIdx.x / LPR, j = threadIdx.x % LPR;
  const int wabs = planar ? j : ftile * LPR + j;        // word index of this lane within a row of bins32
  const int Fl = planar ? F - ftile * FTILE : F;
  const unsigned* bins32 = (const unsigned*)(planar ? bins + (size_t)ftile * (size_t)N * 32 : bins);
  // packed modes have no second plane: sa / sb carry the weight scale and field shift of the packed word
  const float sa = (float)qs[PACKED ? 10 : 0], sb = (float)qs[PACKED ? 12 : 1], sp = (float)qs[4];
  const HistSrc src = make_src(bins32, aw, ay, N, W, lgw);
  // per tile feature: bin count and copies of its bins (NONA: no NA bin, so copies of bins < nb never reach 255)
  __shared__ int srep[FTILE], snb[FTILE], sfine[FTILE];
  if (threadIdx.x < FTILE) {
    const int fg = ftile * FTILE + threadIdx.x;
    const int fi = (fine_f && fg < F) ? fine_f[fg] : 0;
    const int nb = (NONA && nbins_f && fg < F && !fi) ? nbins_f[fg] : 0;
    srep[threadIdx.x] = (nb > 0 && nb * 4 <= NA_BIN) ? 4 : (nb > 0 && nb * 2 <= NA_BIN) ? 2 : 1;
    snb[threadIdx.x] = nb;
    sfine[threadIdx.x] = fi;
  }
  __syncthreads();

  __shared__ Dec spd;
  RowFilter flt{&spd, bins, stride, 0, -1, 0, 0, 0, 0, false};
  int lcnt = 0;
  int cur = -1, since = 0, cur_parent = -1;
  unsigned pre[FNP], pre2[FNP];      // FILT: prefetched split bytes of tiles pre_t and pre2_t
  int pre_t = -1, pre2_t = -1;
  int qn = 0;                        // FILT: rows in this wave's queue (wave-uniform)
  bool acc = false;
  double wyy = 0.0;
  // FILT: histogram the wave's queued rows of the current node (before its LDS histogram is flushed)
  // FILT pipeline state: the batch gathered last (its atomics not yet issued)
  const FiltLane FL = filt_lane<PACKED, UNIT, FINE>(src, W, wabs, Fl, lane >> 3, j, j == 0 && ftile == 0, srep, snb,
                                                    sfine);
  unsigned wdP[8];
  float yP[8], wP[8];
  int np = 0;                        // rows of the pending batch (0: none)
  auto drain = [&]() {
    if (!FILT) return;
    float wf2 = 0.f;
    if (qn > 0) {
      unsigned wdN[8];
      float yN[8], wN[8];
      wave_sync_lds();
      filt_gather<UNIT, BUF>(FL, src, W, wq, qn, lane >> 3, wdN, yN, wN);
      if (np > 0) filt_atoms<PACKED, UNIT, NONA, FINE>(FL, h, nayy, np, lane >> 3, j, wdP, yP, wP, wf2, sa, sb, sp);
      filt_atoms<PACKED, UNIT, NONA, FINE>(FL, h, nayy, qn, lane >> 3, j, wdN, yN, wN, wf2, sa, sb, sp);
      qn = 0;
      wave_sync_lds();
    } else if (np > 0) {
      filt_atoms<PACKED, UNIT, NONA, FINE>(FL, h, nayy, np, lane >> 3, j, wdP, yP, wP, wf2, sa, sb, sp);
    }
    np = 0;
    wyy += (double)wf2;
  };
  auto flush = [&]() {
    drain();
    if (dbg & 1) return;
    double v[4] = {wyy, (double)lcnt, 0, 0};
    block_sum4(v, red);
    __syncthreads();
    const size_t so = (size_t)(blockIdx.x + cur) * slot_doubles;
    flush_partial(h, nayy, v[0], ftile, F, f32 ? (double*)((float*)partials + so) : partials + so, qs, packed, acc,
                  f32 != 0, srep, snb, sfine);
    if (FILT && threadIdx.x == 0 && v[1] != 0.0) atomicAdd(nl_out + cur_parent, (int)v[1]);
    __syncthreads();
  };
  if (!FILT) {
    // plain levels: the block's tiles are runs of whole node ranges — one hist_span per (node, packed window), no
    // per-tile node lookup or per-tile lane setup
    int t = t0;
    while (t < t1) {
      const int node = find_node(tile_prefix, n_nodes, t);
      const Node nd = nodes[node];
      const int tn0 = tile_prefix[node];
      const int te = max(t + 1, min(t1, tile_prefix[node + 1]));
      int rs = nd.start + (t - tn0) * TILE;
      const int re = min(nd.start + nd.len, nd.start + (te - tn0) * TILE);
      t = te;
      if (!nd.build) continue;
      while (rs < re) {
        if (node != cur || (packed && since >= PACK_MAX)) {
          if (cur >= 0) flush();
          acc = node == cur;
          lds_zero64(h, packed ? HPLANE : 2 * HPLANE);
          for (int i = threadIdx.x; i < FTILE; i += blockDim.x) nayy[i] = 0.f;
          wyy = 0.0;
          lcnt = 0;
          since = 0;
          cur = node;
          cur_parent = nd.parent;
          __syncthreads();
        }
        const int we = packed ? min(re, rs + (PACK_MAX - since)) : re;
        float wf = 0.f;
        hist_span<PACKED, UNIT, NONA, BUF, FINE>(h, nayy, src, W, wabs, Fl, j == 0 && ftile == 0, rs, we, g, j, wf, sa,
                                                 sb, sp, srep, snb, sfine, (dbg & 2) != 0);
        wyy += (double)wf;
        since += we - rs;
        rs = we;
      }
    }
  }
  for (int t = FILT ? t0 : t1; t < t1; ++t) {
    const int node = find_node(tile_prefix, n_nodes, t);
    const Node nd = nodes[node];
    if (!nd.build) continue;
    const int r0 = nd.start + (t - tile_prefix[node]) * TILE;
    const int r1 = min(r0 + TILE, nd.start + nd.len);
    // new node, or (packed) the flush window is full: flush the LDS tile and restart it
    if (node != cur || (packed && since + (r1 - r0) > PACK_MAX)) {
      if (cur >= 0) flush();
      acc = node == cur;    // same node, next window: add into the partial stored by the first flush
      lds_zero64(h, packed ? HPLANE : 2 * HPLANE);
      for (int i = threadIdx.x; i < FTILE; i += blockDim.x) nayy[i] = 0.f;
      if (FILT && threadIdx.x < (int)(sizeof(Dec) / 4))
        ((int*)&spd)[threadIdx.x] = ((const int*)(pdec + nd.parent))[threadIdx.x];
      wyy = 0.0;
      lcnt = 0;
      since = 0;
      cur = node;
      cur_parent = nd.parent;
      __syncthreads();
      if (FILT) {
        flt.feat = spd.feat;
        flt.fptr = bins + bin_off(0, spd.feat, stride, N, planar);
        flt.fstride = planar ? 32 : stride;
        if (fdir) { flt.fptr = fdir; flt.fstride = 1; }
        const int jw = (spd.feat >> 2) - ftile * LPR;
        flt.jw = (jw >= 0 && jw < LPR) ? jw : -1;
        flt.dir = nd.dir;
        flt.bin = spd.bin; flt.na_left = spd.na_left; flt.is_cat = spd.is_cat;
        if (fdir) { flt.bin = 1; flt.na_left = 0; flt.is_cat = 0; }    // direction bytes: 0 goes left
        flt.count = ftile == 0;
      }
    }
    since += r1 - r0;
    float wf = 0.f;
    if (FILT) {
      // the split bytes of this tile were prefetched during the previous tile's atomics when both tiles
      // belong to the same node (the common case); a node change loads them here
      // split bytes are prefetched TWO tiles ahead (same node: same filter): the direction loads are this pass's HBM
      // stream (every line of the parent's rows), so a wave keeps two tiles of them in flight behind its atomics
      if (pre_t != t) filt_load(flt, r0, r1, pre);
      unsigned curb[FNP];
#pragma unroll
      for (int k = 0; k < FNP; ++k) curb[k] = pre[k];
      const int nend = nd.start + nd.len;
      const int rn1 = r0 + TILE, rn2 = r0 + 2 * TILE;
      if (pre2_t == t + 1) {
#pragma unroll
        for (int k = 0; k < FNP; ++k) pre[k] = pre2[k];
        pre_t = t + 1;
      } else if (t + 1 < t1 && rn1 < nend) {
        filt_load(flt, rn1, min(rn1 + TILE, nend), pre);
        pre_t = t + 1;
      } else {
        pre_t = -1;
      }
      if (t + 2 < t1 && rn2 < nend) {
        filt_load(flt, rn2, min(rn2 + TILE, nend), pre2);
        pre2_t = t + 2;
      } else {
        pre2_t = -1;
      }
      qn = filt_append(flt, r0, r1, wq, qn, lcnt, curb);
      // full 64-row batches of the wave's queue (8 lane groups x UNR rows); the rest waits for the next tile
      // of this node (or the drain before the flush)
      while (qn >= 64) {
        unsigned wdN[8];
        float yN[8], wN[8];
        wave_sync_lds();
        filt_gather<UNIT, BUF>(FL, src, W, wq, 64, lane >> 3, wdN, yN, wN);   // the next batch's loads go out first
        const int rest = qn - 64;                        // <= 127: move to the queue front (no lane overlap)
        wave_sync_lds();
        const int v0 = lane < rest ? wq[64 + lane] : 0, v1 = lane + 64 < rest ? wq[128 + lane] : 0;
        if (lane < rest) wq[lane] = v0;
        if (lane + 64 < rest) wq[64 + lane] = v1;
        qn = rest;
        if (np > 0) filt_atoms<PACKED, UNIT, NONA, FINE>(FL, h, nayy, np, lane >> 3, j, wdP, yP, wP, wf, sa, sb, sp);
#pragma unroll
        for (int u = 0; u < 8; ++u) { wdP[u] = wdN[u]; yP[u] = yN[u]; wP[u] = wN[u]; }
        np = 64;
      }
    }
    wyy += (double)wf;
  }
  if (cur >= 0) flush();
}

// k_hist_reduce: per build node, sum its partial slots in block order (deterministic fp64) and write
// the node histogram to out[slot] (slot = parent: the compact build buffer; 0 for the root).
// Block b covers tiles [b*per, (b+1)*per), so node n's blocks are b in [bp[n]/per, (bp[n+1]-1)/per] and
// its partials sit at b + n. With hist_next != nullptr (single process) the sibling subtraction is fused:
// hist_next[n] = sum and hist_next[sib] = hist_cur[parent] - sum (no compact-buffer round trip).
#define RW 8   // waves per k_hist_reduce block: wave w sums partials b0 + w, b0 + w + RW, ... of 64 columns
// COLS (levels of many small nodes, fan-in <= ~32 partials): each wave owns 64 columns of its own and sums ALL the
// node's partials of them — no LDS combine, 8x fewer blocks. MEASURED r5: the partial-split form launched
// 225 x 32 blocks at level 5 of the headline tree, 2-3 loads per lane each (14 us for ~36 MB).
template <typename P, typename TO, bool COLS>
__global__ __launch_bounds__(RW * 64) void k_hist_reduce(
    const P* __restrict__ partials, int slot_doubles, int used, const Node* __restrict__ nodes,
    const int* __restrict__ bp, const int* __restrict__ meta, int G, TO* __restrict__ out, int ostride,
    double* __restrict__ hist_next, const double* __restrict__ hist_cur, int lo_F) {
  const int node = blockIdx.y;
  if (node >= meta[0]) return;
  const Node nd = nodes[node];
  if (!nd.build) return;
  __shared__ double red[RW][64];
  const int n_tiles = meta[2];
  const int per = n_tiles > 0 ? (n_tiles + G - 1) / G : 1;
  const int t0 = bp[node], t1 = bp[node + 1];
  const int b0 = t0 / per, b1 = t1 > t0 ? (t1 - 1) / per : b0 - 1;
  const int oslot = nd.parent >= 0 ? nd.parent : 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int i = (COLS ? blockIdx.x * RW + w : blockIdx.x) * 64 + lane;
  if (lo_F > 0) {
    // narrow level: only the entries of columns < lo_F ([bin][lo_F][2] of the [bin][F][2] layout) and the tail
    const int F = (used - 1) / (2 * NBIN + 1), lo2 = 2 * lo_F;
    const int vb = NBIN * lo2;
    if (i >= vb + F + 1) i = used;   // past the virtual range: idle lane
    else i = i < vb ? (i / lo2) * 2 * F + i % lo2 : NBIN * 2 * F + (i - vb);
  }
  const int ic = min(i, used - 1);
  // 8 independent loads in flight per lane (the root's 256 partials: 4 dependent rounds per wave instead of 8);
  // fixed summation order -> deterministic result
  double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  constexpr int ST = COLS ? 1 : RW;     // partial stride of this wave
  int b = b0 + (COLS ? 0 : w);
  for (; b + 7 * ST <= b1; b += 8 * ST) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += (double)partials[(size_t)(b + k * ST + node) * slot_doubles + ic];
  }
  for (; b <= b1; b += ST) a[0] += (double)partials[(size_t)(b + node) * slot_doubles + ic];
  double acc = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  if (!COLS) {
    red[w][lane] = acc;
    __syncthreads();
    if (w != 0) return;
    acc = red[0][lane];
#pragma unroll
    for (int k = 1; k < RW; ++k) acc += red[k][lane];
  }
  if (i >= used) return;
  if (out) out[(size_t)oslot * ostride + i] = (TO)acc;   // the compact build slot (row-sharded: wire dtype)
  if (hist_next) {
    hist_next[(size_t)node * slot_doubles + i] = acc;
    if (nd.sib >= 0)
      hist_next[(size_t)nd.sib * slot_doubles + i] = hist_cur[(size_t)nd.parent * slot_doubles + i] - acc;
  }
}

// ------------------------------------------------------------------------------------------------
// Row-sharded levels: the node histograms are DERIVED inside k_split_find from the exchanged build slots
// (fused sibling subtraction, no separate k_subtract launch): node = build ? recv[parent] : prev[parent] -
// recv[parent]; each (node, feature) block also writes its feature's part of the node slot (the next level
// subtracts from it). recv: [parent][E] in the wire dtype.
struct Derive {
  const void* recv;
  int f32, E;
  const double* prev;      // the previous level's node histograms (slot stride = slot_doubles)
  const Node* nodes;       // this level's node list (parent, build)
};

// a + x * y rounded twice (never contracted into an fma): split points the host reference reproduces bit-exactly
__device__ __forceinline__ double add_mul_rn(double a, double x, double y) {
#pragma clang fp contract(off)
  return a + x * y;
}

// ------------------------------------------------------------------------------------------------
// Wide-categorical group split (H2O's single sort over ALL levels, DTree.java:1004-1013): the group's first column
// block merges the group's real columns into one histogram over the global bins g = 254k + b (k = column, b < its
// 'elsewhere' bin), sorts all of them by mean response (empty bins first, ties by bin), scans every threshold of
// the sorted order and writes one candidate whose bitset covers every level (NBW words). Same rules, order and
// tie breaks as the single-column categorical search above (RefTreeBuilder: ops/tree.py split_find_ref, gcat).
struct HistRead {        // a node histogram entry: the slot, or (row-sharded) derived from the exchanged build slots
  const double* slot;
  const void* recv;
  const double* pv;
  size_t rb;
  int f32, build, derive;
  __device__ __forceinline__ double operator()(size_t i) const {
    if (!derive) return slot[i];
    const double r = f32 ? (double)((const float*)recv)[rb + i] : ((const double*)recv)[rb + i];
    return build ? r : pv[i] - r;
  }
};
#define GBINS 1024
__device__ void split_find_group(const HistRead& hv, int node, int f, int gg, int hs, int FL,
                                 const int* __restrict__ nbins_f, const int* __restrict__ mono_f, const SplitParams& p,
                                 int level, int f0, Cand* __restrict__ cand) {
  __shared__ double gk[GBINS], gw[GBINS], gy[GBINS];
  __shared__ int gi[GBINS];
  __shared__ double gwt[8];
  __shared__ double gbe[4];
  __shared__ int gbc[4];
  __shared__ unsigned gbits[NBW];
  __shared__ int s_lo, s_hi;
  const int t = threadIdx.x;                 // 256 threads, 4 bins each
  int L = 0;
  for (int k = 0; k < gg; ++k) L = 254 * k + (nbins_f[f + k] - 1);
  for (int i = t; i < GBINS; i += 256) {
    const int k = i / 254, b = i - 254 * k;
    double w = 0.0, y = 0.0;
    bool in = false;
    if (k < gg && b < nbins_f[f + k] - 1) {
      in = true;
      w = hv((size_t)b * hs + 2 * (f + k));
      y = hv((size_t)b * hs + 2 * (f + k) + 1);
    }
    gw[i] = w; gy[i] = y;
    gk[i] = in ? (w > 0 ? y / w : -1.0e308) : 1.0e308;
    gi[i] = i;
  }
  if (t < NBW) gbits[t] = 0u;
  __syncthreads();
  // bitonic sort of (key, bin) ascending over the 1024 entries
  for (int k = 2; k <= GBINS; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = t; i < GBINS; i += 256) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const bool up = (i & k) == 0;
          const double a = gk[i], b = gk[ixj];
          const int ia = gi[i], ib = gi[ixj];
          const bool gt = (a > b) || (a == b && ia > ib);
          if (gt == up) { gk[i] = b; gk[ixj] = a; gi[i] = ib; gi[ixj] = ia; }
        }
      }
      __syncthreads();
    }
  }
  // inclusive prefix sums of (w, wy) in sorted order: thread t owns positions 4t .. 4t+3
  double a[4], b[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) { a[j] = gw[gi[4 * t + j]]; b[j] = gy[gi[4 * t + j]]; }
#pragma unroll
  for (int j = 1; j < 4; ++j) { a[j] += a[j - 1]; b[j] += b[j - 1]; }
  {
    const int lane = t & 63, wv = t >> 6;
    double sa = a[3], sb = b[3];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double a2 = __shfl_up(sa, o, 64), b2 = __shfl_up(sb, o, 64);
      if (lane >= o) { sa += a2; sb += b2; }
    }
    if (lane == 63) { gwt[wv] = sa; gwt[4 + wv] = sb; }
    __syncthreads();
    double oa = sa - a[3], ob = sb - b[3];          // exclusive prefix within the wave
    for (int k = 0; k < wv; ++k) { oa += gwt[k]; ob += gwt[4 + k]; }
#pragma unroll
    for (int j = 0; j < 4; ++j) { a[j] += oa; b[j] += ob; }
  }
  __syncthreads();                                  // every gw / gy read done: reuse them as the sorted sums
#pragma unroll
  for (int j = 0; j < 4; ++j) { gw[4 * t + j] = a[j]; gy[4 * t + j] = b[j]; }
  __syncthreads();
  const double* sw = gw;
  const double* swy = gy;
  const double W = sw[GBINS - 1], WY = swy[GBINS - 1];
  const size_t iNA = (size_t)NA_BIN * hs + 2 * f;
  const double wNA = hv(iNA), wyNA = hv(iNA + 1);
  const double naYY = hv((size_t)FL * 2 * NBIN + f), wYY = hv((size_t)FL * 2 * NBIN + FL);
  const double Wall = W + wNA, WYall = WY + wyNA;
  auto E = [&](double ww, double yy) -> double {
    if (p.mode == 1) {
      double g = yy;
      if (p.alpha > 0) g = (g > p.alpha) ? g - p.alpha : (g < -p.alpha ? g + p.alpha : 0.0);
      return g * g / (ww + p.lambda);
    }
    return ww > 0 ? yy * yy / ww : 0.0;
  };
  auto leafv = [&](double ww, double yy) -> double {
    return p.mode == 1 ? yy / (ww + p.lambda) : (ww > 0 ? yy / ww : 0.0);
  };
  const double min_w = p.min_w;
  const int mono = mono_f ? mono_f[f] : 0;
  const bool random_mode = p.random_split != 0;
  int rand_b = -1;
  if (random_mode) {
    if (t == 0) { s_lo = 0; s_hi = -1; }
    __syncthreads();
    for (int j = 0; j < 4; ++j) {
      const int q = 4 * t + j;
      const double cw = sw[q], pw = q > 0 ? sw[q - 1] : 0.0;
      if (q < L && cw > 0 && pw == 0) s_lo = q;
      if (q < L && W > 0 && cw == W && pw < W) s_hi = q;
    }
    __syncthreads();
    if (s_hi > s_lo) {
      const unsigned long long hsh = splitmix64(p.seed ^ ((unsigned long long)level << 48) ^
                                                ((unsigned long long)node << 20) ^ (unsigned long long)(f + f0));
      rand_b = s_lo + 1 + (int)(hsh % (unsigned long long)(s_hi - s_lo));
    }
  }
  double my_e = -1.0e300;
  int my_code = -1;
  for (int j = 0; j < 4; ++j) {
    const int q = 4 * t + j;                        // threshold: sorted positions < q go left
    if (q < 1 || q >= L || (random_mode && q != rand_b)) continue;
    const double wb = sw[q] - sw[q - 1];
    if (!(wb != 0.0 || random_mode)) continue;
    const double wlo = sw[q - 1], wylo = swy[q - 1];
    const double whi = W - wlo, wyhi = WY - wylo;
    double ce = -1.0e300;
    int cc = -1;
    if (wNA == 0.0) {
      if (wlo >= min_w && whi >= min_w) {
        const double e = E(wlo, wylo) + E(whi, wyhi);
        const bool ok = mono == 0 || (mono * leafv(wlo, wylo) <= mono * leafv(whi, wyhi));
        if (ok) { ce = e; cc = q * 2 + (wlo > whi ? 1 : 0); }
      }
    } else {
      if (wlo + wNA >= min_w && whi >= min_w) {
        const double e = E(wlo + wNA, wylo + wyNA) + E(whi, wyhi);
        const bool ok = mono == 0 || (mono * leafv(wlo + wNA, wylo + wyNA) <= mono * leafv(whi, wyhi));
        if (ok && e > ce) { ce = e; cc = q * 2 + 1; }
      }
      if (wlo >= min_w && whi + wNA >= min_w) {
        const double e = E(wlo, wylo) + E(whi + wNA, wyhi + wyNA);
        const bool ok = mono == 0 || (mono * leafv(wlo, wylo) <= mono * leafv(whi + wNA, wyhi + wyNA));
        if (ok && e > ce) { ce = e; cc = q * 2 + 0; }
      }
    }
    if (cc >= 0 && (my_code < 0 || ce > my_e || (ce == my_e && cc < my_code))) { my_e = ce; my_code = cc; }
  }
  if (t == 0 && wNA >= min_w && W > 0 && !random_mode) {     // NA vs REST: the incumbent, wins ties
    const double e = E(W, WY) + E(wNA, wyNA);
    if (my_code < 0 || e > my_e || e == my_e) { my_e = e; my_code = 0; }
  }
  {
    const int lane = t & 63, wv = t >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double e2 = __shfl_xor(my_e, o, 64);
      const int c2 = __shfl_xor(my_code, o, 64);
      if (c2 >= 0 && (my_code < 0 || e2 > my_e || (e2 == my_e && c2 < my_code))) { my_e = e2; my_code = c2; }
    }
    if (lane == 0) { gbe[wv] = my_e; gbc[wv] = my_code; }
    __syncthreads();
    if (t == 0) {
      for (int k = 1; k < 4; ++k) {
        const double e2 = gbe[k];
        const int c2 = gbc[k];
        if (c2 >= 0 && (gbc[0] < 0 || e2 > gbe[0] || (e2 == gbe[0] && c2 < gbc[0]))) { gbe[0] = e2; gbc[0] = c2; }
      }
    }
    __syncthreads();
  }
  const int code = gbc[0];
  const double be = gbe[0];
  int bsp = 0, nal = 0;
  if (code > 0) { bsp = code >> 1; nal = code & 1; }
  if (code > 0) {
    for (int j = 0; j < 4; ++j) {
      const int q = 4 * t + j;
      if (q >= L) continue;
      const int cidx = gi[q];
      const bool empty = (sw[q] - (q > 0 ? sw[q - 1] : 0.0)) == 0.0;
      const bool left = empty ? (nal != 0) : (q < bsp);
      if (left) atomicOr(&gbits[cidx >> 5], 1u << (cidx & 31));
    }
  }
  __syncthreads();
  if (t == 0) {
    int valid = 0;
    double wl = 0, wr = 0, yl = 0, yr = 0;
    if (code == 0) { wl = W; yl = WY; wr = wNA; yr = wyNA; }
    else if (code > 0) {
      wl = sw[bsp - 1]; yl = swy[bsp - 1]; wr = W - wl; yr = WY - yl;
      if (nal) { wl += wNA; yl += wyNA; } else { wr += wNA; yr += wyNA; }
    }
    const double Epar = E(Wall, WYall);
    double gain = be - Epar;
    if (code >= 0 && Wall >= 2.0 * min_w) {
      if (p.mode == 0) {
        const double var = wYY * Wall - WYall * WYall;
        const double seBefore = (wNA >= min_w) ? (wYY - Epar) : ((wYY - naYY) - E(W, WY));
        const double seAfter = wYY - be;
        const float pl = (float)(yl / wl), pr = (float)(yr / wr);
        valid = ((float)var != 0.f) && (seAfter < seBefore * (1.0 - p.min_split_improvement)) &&
                (pl != pr) && wl >= min_w && wr >= min_w;
        if (random_mode) valid = wl > 0 && wr > 0;
      } else if (p.mode == 1) {
        valid = (0.5 * gain - p.gamma) > 1e-6 && wl >= min_w && wr >= min_w;
        gain = 0.5 * gain - p.gamma;
      } else {
        valid = wl > 0 && wr > 0;
      }
    }
    unsigned pack = 0u;
    for (int k = 0; k < gg; ++k) pack |= (unsigned)(nbins_f[f + k] - 1) << (8 * k);
    Cand* c = cand + (size_t)node * FL + f;
    c->expl = be; c->gain = gain; c->wl = wl; c->wr = wr;
    c->predl = (float)leafv(wl, yl); c->predr = (float)leafv(wr, yr);
    c->bin = (int)pack;
    c->na_left = (code == 0) ? 0 : nal;
    c->valid = valid;
    c->is_cat = GROUP_CAT;
  }
  if (t < NBW) cand[(size_t)node * FL + f].bits[t] = code == 0 ? 0xFFFFFFFFu : gbits[t];
}

// k_split_find: best split point per (node, feature). grid = (C, F), block 256 (thread = bin).
template <bool GRP>
__device__ __forceinline__ void split_find_body(
    double* __restrict__ hist, int slot_doubles, const int* __restrict__ meta, int F,
    const int* __restrict__ nbins_f, const int* __restrict__ iscat_f, const int* __restrict__ mono_f,
    SplitParams p, int level, Cand* __restrict__ cand, double* __restrict__ root_w,
    const float* __restrict__ edges /*[F][255] global bin edges (inf padded) or null*/, int adapt_nb, int f0,
    int FL, Derive dv) {
  // f0: global id of this launch's first feature (feature-sliced row-sharded runs search only the rank's
  // slice; per-feature arrays arrive offset by f0). FL: features of the slot LAYOUT and of the cand row
  // stride (the slice width Fs, >= the F features searched here; F everywhere else)
  const int node = blockIdx.x, f = blockIdx.y, t = threadIdx.x;
  if (node >= meta[0]) return;
  if (p.fcut > 0 && f + f0 >= p.fcut) {     // a column this level does not search (its histogram is not built)
    if (t == 0) cand[(size_t)node * FL + f].valid = 0;
    return;
  }
  __shared__ double sw[256], swy[256], skey[256];
  __shared__ int sidx[256];
  __shared__ double best_e[256];
  __shared__ int best_i[256];

  double* slot = hist + (size_t)node * slot_doubles;
  const int hs = 2 * FL;
  const int nb = nbins_f[f];
  const bool cat = iscat_f[f] != 0;
  const int mono = mono_f ? mono_f[f] : 0;
  const size_t iNA = (size_t)NA_BIN * hs + 2 * f, iT = (size_t)t * hs + 2 * f;
  const size_t iNY = (size_t)FL * 2 * NBIN + f, iWY = (size_t)FL * 2 * NBIN + FL;
  double wNA, wyNA, naYY, wYY, w = 0, wy = 0;
  if (dv.recv) {
    const Node nd = dv.nodes[node];
    const int ps = nd.parent < 0 ? 0 : nd.parent;
    const size_t rb = (size_t)ps * dv.E;
    const double* pv = dv.prev + (size_t)ps * slot_doubles;
    auto ld = [&](size_t i) -> double {
      const double r = dv.f32 ? (double)((const float*)dv.recv)[rb + i] : ((const double*)dv.recv)[rb + i];
      return nd.build ? r : pv[i] - r;
    };
    wNA = ld(iNA); wyNA = ld(iNA + 1); naYY = ld(iNY); wYY = ld(iWY);
    const double a = ld(iT), b = ld(iT + 1);
    slot[iT] = a; slot[iT + 1] = b;                      // this feature's bins (NA included: t = NA_BIN)
    if (t == 0) { slot[iNY] = naYY; if (f == 0) slot[iWY] = wYY; }
    if (t < nb && t < NA_BIN) { w = a; wy = b; }
  } else {
    wNA = slot[iNA]; wyNA = slot[iNA + 1]; naYY = slot[iNY]; wYY = slot[iWY];
    if (t < nb && t < NA_BIN) { w = slot[iT]; wy = slot[iT + 1]; }
  }
  if (GRP && p.gcat) {
    const int gg = p.gcat[f + f0];
    if (gg < 0) {                       // a group member or padding column: the group's first column searches it
      if (t == 0) {
        Cand* c = cand + (size_t)node * FL + f;
        c->valid = 0; c->expl = -1.0e300; c->is_cat = 0;
      }
      return;
    }
    if (gg > 0) {
      HistRead hr{slot, dv.recv, nullptr, 0, dv.f32, 1, dv.recv != nullptr ? 1 : 0};
      if (dv.recv) {
        const Node nd = dv.nodes[node];
        const int ps = nd.parent < 0 ? 0 : nd.parent;
        hr.rb = (size_t)ps * dv.E;
        hr.pv = dv.prev + (size_t)ps * slot_doubles;
        hr.build = nd.build;
      }
      split_find_group(hr, node, f, gg, hs, FL, nbins_f, mono_f, p, level, f0, cand);
      return;
    }
  }
  sidx[t] = t;
  if (cat) {
    // sort bins by mean response (empty bins first, out-of-range bins last) — DTree.java:1006
    skey[t] = (t < nb) ? (w > 0 ? wy / w : -1.0e308) : 1.0e308;
    sw[t] = w; swy[t] = wy;
    __syncthreads();
    for (int k = 2; k <= 256; k <<= 1) {
      for (int jj = k >> 1; jj > 0; jj >>= 1) {
        const int ixj = t ^ jj;
        if (ixj > t) {
          const bool up = ((t & k) == 0);
          const double a = skey[t], b = skey[ixj];
          const int ia = sidx[t], ib = sidx[ixj];
          const bool gt = (a > b) || (a == b && ia > ib);
          if (gt == up) { skey[t] = b; skey[ixj] = a; sidx[t] = ib; sidx[ixj] = ia; }
        }
        __syncthreads();
      }
    }
    w = sw[sidx[t]]; wy = swy[sidx[t]];
    __syncthreads();
  }
  // inclusive scan of (w, wy) in sorted order: per-wave shuffle scans + the previous waves' totals (two
  // barriers instead of sixteen). Histogram entries are fixed-point multiples of one quantum, so every
  // summation order gives the same fp64 sums.
  {
    const int lane = t & 63, wv = t >> 6;
    double a = w, b = wy;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const double a2 = __shfl_up(a, o, 64), b2 = __shfl_up(b, o, 64);
      if (lane >= o) { a += a2; b += b2; }
    }
    __shared__ double wtot[8];
    if (lane == 63) { wtot[wv] = a; wtot[4 + wv] = b; }
    __syncthreads();
    for (int k = 0; k < wv; ++k) { a += wtot[k]; b += wtot[4 + k]; }
    sw[t] = a; swy[t] = b;
    __syncthreads();
  }
  const double W = sw[255], WY = swy[255];
  const double Wall = W + wNA, WYall = WY + wyNA;
  if (root_w && node == 0 && f + f0 == 0 && t == 0) *root_w = Wall;   // level 0: the tree's total weight

  auto E = [&](double ww, double yy) -> double {
    if (p.mode == 1) {
      double g = yy;  // stat is -sum(g): T_alpha soft-threshold
      if (p.alpha > 0) g = (g > p.alpha) ? g - p.alpha : (g < -p.alpha ? g + p.alpha : 0.0);
      return g * g / (ww + p.lambda);
    }
    return ww > 0 ? yy * yy / ww : 0.0;
  };
  auto leafv = [&](double ww, double yy) -> double {
    return p.mode == 1 ? yy / (ww + p.lambda) : (ww > 0 ? yy / ww : 0.0);
  };

  // candidate of this thread: threshold b = t (left = sorted positions < t)
  double my_e = -1.0e300;
  int my_code = -1;  // code = b*2 + na_left (b in 1..nb-1), or 0 for NA-vs-rest
  const double min_w = p.min_w;
  const bool random_mode = p.random_split != 0;
  int rand_b = -1;
  if (random_mode) {
    // random threshold strictly inside the node's occupied bin range [lo, hi] (isolation / XRT):
    // lo = first non-empty sorted position, hi = last; b in (lo, hi] keeps both sides non-empty
    __shared__ int s_lo, s_hi;
    if (t == 0) { s_lo = 0; s_hi = -1; }
    __syncthreads();
    const double cw = sw[t], pw = t > 0 ? sw[t - 1] : 0.0;
    if (t < nb && cw > 0 && pw == 0) s_lo = t;
    if (t < nb && W > 0 && cw == W && pw < W) s_hi = t;
    __syncthreads();
    if (s_hi > s_lo) {
      unsigned long long hsh = splitmix64(p.seed ^ ((unsigned long long)level << 48) ^
                                          ((unsigned long long)node << 20) ^ (unsigned long long)(f + f0));
      rand_b = s_lo + 1 + (int)(hsh % (unsigned long long)(s_hi - s_lo));
    }
  }
  // Numeric candidate lattice of the histogram type (DHistogram / DTree), over the node's occupied value range
  // [lo, hi] on the global-bin lattice: a threshold t ("bins < t go left" = x < edge[t-1]) is kept iff one of
  // the type's split points falls in (edge[t-2], edge[t-1]]. adapt_nb = max(nbins, nbins_top_level >> level).
  //  UniformAdaptive: adapt_nb - 1 uniform cut points (the H2O default).
  //  Random: adapt_nb - 1 uniformly random cut points (DHistogram.makeRandomSplitPoints).
  //  UniformRobust: UniformAdaptive, unless <= 20% of the uniform cells hold data; then GuidedSplitPoints:
  //    the non-empty cells are kept and refined uniformly, the freed budget adapt_nb - K - 2 handed out in
  //    ceil(budget * share) portions by descending cell share (DTree.java:398-409). The share is the cell's
  //    weight: the 2-statistic histogram has no per-bin sum of squares for the reference's per-bin SE.
  //  RoundRobin: one of {AUTO, UniformAdaptive, Random, QuantilesGlobal} per (node, feature), drawn from
  //    the tree seed (DHistogram.java:226-229).
  int lt = (adapt_nb > 1 && edges != nullptr && !cat && !random_mode) ? p.hist_type : HT_QUANTILES;
  if (lt == HT_ROUND_ROBIN) {
    const unsigned r = (unsigned)(splitmix64(p.seed ^ 0xDECAFull ^ ((unsigned long long)level << 48) ^
                                             ((unsigned long long)node << 20) ^ (unsigned long long)(f + f0)) & 3ull);
    lt = r == 3 ? HT_QUANTILES : (r == 2 ? HT_RANDOM : HT_UNIFORM);
  }
  bool lattice_ok = true;
  if (lt != HT_QUANTILES) {
    __shared__ int a_lo, a_hi, s_guided;
    __shared__ unsigned char smark[256];
    if (t == 0) { a_lo = 0; a_hi = -1; s_guided = 0; }
    smark[t] = 0;
    __syncthreads();
    const double cw = sw[t], pw = t > 0 ? sw[t - 1] : 0.0;
    if (t < nb && cw > 0 && pw == 0) a_lo = t;
    if (t < nb && W > 0 && cw == W && pw < W) a_hi = t;
    __shared__ int r_lo, r_hi;
    const bool ranged = p.range_on != 0;
    if (ranged) {
      // the observed range the node bins over: its own at the root, its parent's below (the parent's slot of the
      // previous level's histograms, this column's data bins)
      if (t == 0) { r_lo = 1 << 30; r_hi = -1; }
      __syncthreads();
      const Node* rn = p.rnodes ? p.rnodes + node : nullptr;
      const bool up = level > 0 && rn != nullptr && rn->parent >= 0 && p.hprev != nullptr;
      if (up) {
        const double pwt = (t < nb && t < NA_BIN) ? p.hprev[(size_t)rn->parent * slot_doubles + (size_t)t * hs + 2 * f]
                                                  : 0.0;
        if (pwt > 0) { atomicMin(&r_lo, t); atomicMax(&r_hi, t); }
      } else if (t < nb && t < NA_BIN && w > 0) {
        atomicMin(&r_lo, t); atomicMax(&r_hi, t);
      }
    }
    __syncthreads();
    const float* e = edges + (size_t)f * 255;
    if (a_hi > a_lo && (ranged || lt == HT_RANDOM || a_hi - a_lo + 1 > adapt_nb)) {
      double lo = (double)e[a_lo > 0 ? a_lo - 1 : 0];
      double hi = (double)e[a_hi <= nb - 2 ? a_hi : nb - 2];
      if (ranged) {
        const int gf = f + f0;
        if (r_hi < 0) {
          lo = hi = 0.0;                              // the parent saw no value of this column: no lattice cut
        } else {
          lo = r_lo > 0 ? (double)e[r_lo - 1] : (double)p.vrange[2 * gf];
          hi = r_hi < nb - 1 ? (double)e[r_hi] : (double)p.vrange[2 * gf + 1];
          const Node* rn = p.rnodes ? p.rnodes + node : nullptr;
          if (level > 0 && rn != nullptr && rn->parent >= 0 && p.pdec != nullptr) {
            const Dec& pd = p.pdec[rn->parent];
            const bool same = p.fgroup ? ((p.fgroup[gf] & 0x3FFFFFFF) == (p.fgroup[pd.feat] & 0x3FFFFFFF))
                                       : (pd.feat == gf);
            if (pd.feat >= 0 && !pd.is_cat && pd.bin != NA_BIN && pd.bin > 0 && same) {
              const double v = (double)p.edges_all[(size_t)pd.feat * 255 + pd.bin - 1];
              if (rn->dir == 0) hi = hi < v ? hi : v;
              else lo = lo > v ? lo : v;
            }
          }
        }
      }
      if (hi > lo) {
        const double sc = (double)adapt_nb / (hi - lo);
        auto cnt = [&](double x) -> int {
          double c = floor((x - lo) * sc);
          return (int)(c < 0 ? 0 : (c > adapt_nb - 1 ? adapt_nb - 1 : c));
        };
        // a split point x marks threshold t = 1 + (first i with edge[i] >= x), t <= nb - 1
        auto mark = [&](double x) {
          int a = 0, b = nb - 1;
          while (a < b) { const int m = (a + b) >> 1; if ((double)e[m] >= x) b = m; else a = m + 1; }
          if (a < nb - 1) smark[a + 1] = 1;
        };
        if (lt == HT_ROBUST) {
          // cells (adapt_nb < 256 here) of the uniform lattice: bin t's lower edge lies in cell(t); the
          // bins of one cell are contiguous, so a cell's weight is a difference of the prefix sums
          __shared__ int cstart[256];
          __shared__ double cwt[256];
          __shared__ int s_k;
          if (t == 0) s_k = 0;
          cwt[t] = 0.0;
          __syncthreads();
          const int ci = (t >= a_lo && t <= a_hi) ? (t == a_lo ? 0 : cnt((double)e[t - 1])) : -1;
          const int cprev = (t > a_lo && t <= a_hi) ? (t - 1 == a_lo ? 0 : cnt((double)e[t - 2])) : -1;
          if (ci >= 0 && ci != cprev) cstart[ci] = t;
          __syncthreads();
          const int cnext = (t >= a_lo && t < a_hi) ? cnt((double)e[t]) : -1;
          if (ci >= 0 && ci != cnext) {
            const double wc = sw[t] - (cstart[ci] > 0 ? sw[cstart[ci] - 1] : 0.0);
            cwt[ci] = wc;
            if (wc > 0) atomicAdd(&s_k, 1);
          }
          __syncthreads();
          const int K = s_k;
          const int budget = adapt_nb - K - 2;
          if ((double)K <= 0.2 * (double)adapt_nb && budget > 0 && K > 0) {
            // rank of this cell in descending weight (ties: lower cell first), then the budget prefix
            const double mw = t < adapt_nb ? cwt[t] : 0.0;
            __shared__ int qv[256];
            __shared__ int rk[256];
            int q = 0, r = 0;
            if (mw > 0) {
              q = (int)ceil((double)budget * mw / W);
              for (int c = 0; c < adapt_nb; ++c) {
                const double oc = cwt[c];
                r += (oc > mw || (oc == mw && c < t)) ? 1 : 0;
              }
            }
            qv[t] = q; rk[t] = mw > 0 ? r : 1 << 20;
            __syncthreads();
            if (mw > 0) {
              int before = 0;
              for (int c = 0; c < adapt_nb; ++c) before += (rk[c] < r) ? qv[c] : 0;
              const int left = budget - before;
              const int nnew = left <= 0 ? 0 : (q < left ? q : left);
              const double step = (hi - lo) / (double)adapt_nb;
              const double c0 = add_mul_rn(lo, step, (double)t);
              const double sub = step / (double)(1 + nnew);
              for (int j = 0; j <= nnew; ++j) mark(add_mul_rn(c0, sub, (double)j));
            }
            if (t == 0) { mark(lo); mark(hi); s_guided = 1; }
          }
          __syncthreads();
          if (!s_guided) lt = HT_UNIFORM;
        }
        if (lt == HT_UNIFORM) {
          lattice_ok = t >= 1 && t < nb && cnt((double)e[t - 1]) > (t >= 2 ? cnt((double)e[t - 2]) : 0);
        } else {
          if (lt == HT_RANDOM) {
            for (int k = 1 + t; k < adapt_nb; k += 256) {
              const unsigned long long h = splitmix64(p.seed ^ 0xC0FFEEull ^ ((unsigned long long)level << 48) ^
                                                      ((unsigned long long)node << 20) ^
                                                      ((unsigned long long)(f + f0) << 10) ^ (unsigned long long)k);
              mark(add_mul_rn(lo, hi - lo, (double)(h >> 11) * 0x1p-53));
            }
          }
          __syncthreads();
          lattice_ok = t >= 1 && t < nb && smark[t] != 0;
        }
      }
    }
  }
  if (t >= 1 && t < nb && lattice_ok && (!random_mode || t == rand_b)) {
    const double wb = (t < 256) ? (sw[t] - sw[t - 1]) : 0.0;
    if (wb != 0.0 || random_mode) {
      const double wlo = sw[t - 1], wylo = swy[t - 1];
      const double whi = W - wlo, wyhi = WY - wylo;
      if (wNA == 0.0) {
        if (wlo >= min_w && whi >= min_w) {
          const double e = E(wlo, wylo) + E(whi, wyhi);
          const bool ok = mono == 0 || (mono * leafv(wlo, wylo) <= mono * leafv(whi, wyhi));
          if (ok) { my_e = e; my_code = t * 2 + (wlo > whi ? 1 : 0); }
        }
      } else {
        if (wlo + wNA >= min_w && whi >= min_w) {  // NA left
          const double e = E(wlo + wNA, wylo + wyNA) + E(whi, wyhi);
          const bool ok = mono == 0 || (mono * leafv(wlo + wNA, wylo + wyNA) <= mono * leafv(whi, wyhi));
          if (ok && e > my_e) { my_e = e; my_code = t * 2 + 1; }
        }
        if (wlo >= min_w && whi + wNA >= min_w) {  // NA right
          const double e = E(wlo, wylo) + E(whi + wNA, wyhi + wyNA);
          const bool ok = mono == 0 || (mono * leafv(wlo, wylo) <= mono * leafv(whi + wNA, wyhi + wyNA));
          if (ok && e > my_e) { my_e = e; my_code = t * 2 + 0; }
        }
      }
    }
  }
  // NA vs REST is the incumbent (DTree.java:1140) and wins ties
  if (t == 0 && wNA >= min_w && W > 0 && !random_mode) {
    my_e = E(W, WY) + E(wNA, wyNA);
    my_code = 0;
  }
  // best candidate: larger explained wins; ties -> smaller threshold code (code 0 = NA-vs-rest first). A total
  // order, so the wave-shuffle tree and the cross-wave step pick what any reduction order would.
  {
    const int lane = t & 63, wv = t >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double e2 = __shfl_xor(my_e, o, 64);
      const int c2 = __shfl_xor(my_code, o, 64);
      if (c2 >= 0 && (my_code < 0 || e2 > my_e || (e2 == my_e && c2 < my_code))) { my_e = e2; my_code = c2; }
    }
    if (lane == 0) { best_e[wv] = my_e; best_i[wv] = my_code; }
    __syncthreads();
    if (t == 0) {
      for (int k = 1; k < 4; ++k) {
        const double e2 = best_e[k];
        const int c2 = best_i[k];
        if (c2 >= 0 && (best_i[0] < 0 || e2 > best_e[0] || (e2 == best_e[0] && c2 < best_i[0]))) {
          best_e[0] = e2; best_i[0] = c2;
        }
      }
    }
    __syncthreads();
  }
  const int code = best_i[0];
  const double be = best_e[0];
  Cand* c = cand + (size_t)node * FL + f;
  // categorical bitset: left set = sorted positions < b (empty bins follow the NA direction)
  __shared__ unsigned sbits[8];
  if (t < 8) sbits[t] = 0u;
  __syncthreads();
  int b = 0, nal = 0;
  if (code > 0) { b = code >> 1; nal = code & 1; }
  if (cat && code > 0) {
    if (t < nb) {
      const int cidx = sidx[t];
      const bool empty = (sw[t] - (t > 0 ? sw[t - 1] : 0.0)) == 0.0;
      const bool left = empty ? (nal != 0) : (t < b);
      if (left) atomicOr(&sbits[cidx >> 5], 1u << (cidx & 31));
    }
  }
  __syncthreads();
  if (t == 0) {
    int valid = 0;
    double wl = 0, wr = 0, yl = 0, yr = 0;
    if (code == 0) { wl = W; yl = WY; wr = wNA; yr = wyNA; }
    else if (code > 0) {
      wl = sw[b - 1]; yl = swy[b - 1]; wr = W - wl; yr = WY - yl;
      if (nal) { wl += wNA; yl += wyNA; } else { wr += wNA; yr += wyNA; }
    }
    const double Epar = E(Wall, WYall);
    double gain = be - Epar;
    if (code >= 0 && Wall >= 2.0 * min_w) {
      if (p.mode == 0) {
        const double var = wYY * Wall - WYall * WYall;
        const double seBefore = (wNA >= min_w) ? (wYY - Epar) : ((wYY - naYY) - E(W, WY));
        const double seAfter = wYY - be;
        const float pl = (float)(yl / wl), pr = (float)(yr / wr);
        valid = ((float)var != 0.f) && (seAfter < seBefore * (1.0 - p.min_split_improvement)) &&
                (pl != pr) && wl >= min_w && wr >= min_w;
        if (random_mode) valid = wl > 0 && wr > 0;
      } else if (p.mode == 1) {
        valid = (0.5 * gain - p.gamma) > 1e-6 && wl >= min_w && wr >= min_w;
        gain = 0.5 * gain - p.gamma;
      } else {
        valid = wl > 0 && wr > 0;
      }
    }
    c->expl = be; c->gain = gain; c->wl = wl; c->wr = wr;
    c->predl = (float)leafv(wl, yl); c->predr = (float)leafv(wr, yr);
    c->bin = (code == 0) ? NA_BIN : b;
    c->na_left = (code == 0) ? 0 : nal;
    c->valid = valid;
    c->is_cat = cat ? 1 : 0;
  }
  // the bitset: one word per thread (NA vs REST on a categorical: every level left)
  if (t < NBW) c->bits[t] = (cat && code == 0) ? 0xFFFFFFFFu : ((cat && t < 8) ? sbits[t] : 0u);
}

// Best feature of one node (one wave; lane = threadIdx.x & 63): k_split_reduce, and k_plan's prologue on
// levels of at most PLAN_REDUCE_MAX nodes (the single plan block's 16 waves take the nodes; no extra launch).
// fgroup (nullable): engine column -> original feature in bits 0-29; bit 30 set = not the feature's first
// column. A numeric feature binned wider than one byte holds several engine columns (interleaved edge subsets,
// see ops/binning.py); column sampling draws ORIGINAL features (key and rank of a column = its feature's), so
// such a feature is in or out as a whole.
// cfs > 0: cand is the RANK-MAJOR all-gather of a feature-sliced run, [W][ccap][cfs] (rank r searched
// features r*cfs ..), read in place instead of being permuted into [cap][F] first.
__device__ __forceinline__ const Cand& cand_at(const Cand* __restrict__ cand, int node, int f, int F, int cfs,
                                               int ccap) {
  if (cfs > 0) return cand[((size_t)(f / cfs) * ccap + node) * cfs + f % cfs];
  return cand[(size_t)node * F + f];
}

__device__ void reduce_node(const Cand* __restrict__ cand, int node, int F, const int* __restrict__ feat_ok, int k_cols,
                            unsigned long long seed, int level, Dec* __restrict__ dec,
                            const unsigned char* __restrict__ node_ok, const int* __restrict__ fgroup, int lane,
                            int cfs = 0, int ccap = 0) {
  const unsigned char* nok = node_ok ? node_ok + (size_t)node * F : nullptr;
  auto usable = [&](int f) { return feat_ok[f] != 0 && (!nok || nok[f] != 0); };
  auto gid = [&](int f) { return fgroup ? (fgroup[f] & 0x3FFFFFFF) : f; };
  auto leader = [&](int f) { return !fgroup || (fgroup[f] & 0x40000000) == 0; };
  const unsigned long long base = splitmix64(seed ^ ((unsigned long long)(level + 1) << 40) ^ (unsigned long long)node);
  int n_ok = 0;
  for (int f = lane; f < F; f += 64) n_ok += (usable(f) && leader(f)) ? 1 : 0;
  n_ok = wave_sum_i(n_ok);
  const bool sample = k_cols > 0 && k_cols < n_ok;
  double be = -1.0e300;
  int bf = -1;
  for (int f = lane; f < F; f += 64) {
    if (!usable(f)) continue;
    if (sample) {
      const int gf = gid(f);
      const unsigned long long kf = splitmix64(base + (unsigned long long)gf);
      int rank = 0;
      for (int g2 = 0; g2 < F; ++g2) {
        if (!usable(g2) || !leader(g2)) continue;
        const unsigned long long kg = splitmix64(base + (unsigned long long)gid(g2));
        rank += (kg < kf || (kg == kf && gid(g2) < gf)) ? 1 : 0;
      }
      if (rank >= k_cols) continue;
    }
    const Cand& c = cand_at(cand, node, f, F, cfs, ccap);
    if (c.valid && (bf < 0 || c.expl > be)) { be = c.expl; bf = f; }
  }
  // wave argmax, ties -> smaller feature index
  for (int o = 32; o > 0; o >>= 1) {
    const double e2 = __shfl_xor(be, o, 64);
    const int f2 = __shfl_xor(bf, o, 64);
    if (f2 >= 0 && (bf < 0 || e2 > be || (e2 == be && f2 < bf))) { be = e2; bf = f2; }
  }
  Dec* dn = dec + node;
  if (lane == 0) {
    dn->feat = bf;
    if (bf >= 0) {
      const Cand& c = cand_at(cand, node, bf, F, cfs, ccap);
      dn->bin = c.bin; dn->na_left = c.na_left; dn->is_cat = c.is_cat;
      dn->gain = c.gain; dn->wl = c.wl; dn->wr = c.wr; dn->predl = c.predl; dn->predr = c.predr;
    } else {
      dn->bin = 0; dn->na_left = 0; dn->is_cat = 0;
      dn->gain = 0; dn->wl = 0; dn->wr = 0; dn->predl = 0; dn->predr = 0;
    }
  }
  // the bitset: one word per lane (bf is wave-uniform after the argmax)
  if (lane < NBW) dn->bits[lane] = bf >= 0 ? cand_at(cand, node, bf, F, cfs, ccap).bits[lane] : 0u;
}

__global__ __launch_bounds__(64) void k_split_reduce(
    const Cand* __restrict__ cand, const int* __restrict__ meta, int F,
    const int* __restrict__ feat_ok /*[F] per-tree mask, 1 = usable*/, int k_cols,
    unsigned long long seed, int level, Dec* __restrict__ dec,
    const unsigned char* __restrict__ node_ok /*[nodes][F] interaction-constraint mask or null*/,
    const int* __restrict__ fgroup, int cfs, int ccap) {
  const int node = blockIdx.x;
  if (node >= meta[0]) return;
  reduce_node(cand, node, F, feat_ok, k_cols, seed, level, dec, node_ok, fgroup, threadIdx.x, cfs, ccap);
}

struct PlanReduce {          // k_plan's fused k_split_reduce (cand == null: decisions already made)
  const Cand* cand;
  int F;
  const int* feat_ok;
  int k_cols;
  unsigned long long seed;
  const unsigned char* node_ok;
  const int* fgroup;
  int cfs, ccap;             // rank-major sliced candidates (see cand_at); 0 = [cap][F]
  int no_wave;               // 1: levels of <= 64 nodes take the block plan too (H2O_PLAN_WAVE=0)
};
#define PLAN_REDUCE_MAX 256

// ------------------------------------------------------------------------------------------------
// Block-wide exclusive scan helper for k_plan (1024 threads, int values). Returns exclusive prefix
// of `v` for this thread and writes the block total into *total.
__device__ int block_excl_scan(int v, int* sh /*>=17*/, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int w = 0; w < nw; ++w) { const int tmp = sh[w]; sh[w] = s; s += tmp; }
    sh[16] = s;
  }
  __syncthreads();
  const int res = x - v + sh[wid];
  *total = sh[16];
  __syncthreads();
  return res;
}

// Tile prefix of a level's node list: every node owns ceil(len/TILE) tiles (tp); build nodes also
// own tiles in the build prefix (bp) that k_hist_build walks. meta: [0]=nodes [1]=tiles [2]=build tiles.
__device__ void level_tile_prefix(const Node* __restrict__ next, int nn, int* __restrict__ tp,
                                  int* __restrict__ bp, int* __restrict__ meta, int* sh) {
  const int T = blockDim.x, tid = threadIdx.x;
  const int per = (nn + T - 1) / T;
  const int a = min(nn, tid * per), b = min(nn, a + per);
  int s = 0, sbt = 0;
  for (int i = a; i < b; ++i) {
    const int k = (next[i].len + TILE - 1) / TILE;
    s += k;
    sbt += next[i].build ? k : 0;
  }
  int total, totalb;
  int off = block_excl_scan(s, sh, &total);
  int offb = block_excl_scan(sbt, sh, &totalb);
  for (int i = a; i < b; ++i) {
    const int k = (next[i].len + TILE - 1) / TILE;
    tp[i] = off; off += k;
    bp[i] = offb; offb += next[i].build ? k : 0;
  }
  if (tid == 0) {
    tp[nn] = total; bp[nn] = totalb;
    meta[0] = nn; meta[1] = total; meta[2] = totalb;
  }
}

// k_plan: one block. Numbers the children of a level (compacted, capacity-limited) and the new
// leaves, chooses which child is histogrammed (the lighter one by GLOBAL weight, so every rank of a
// row-sharded run plans alike) and writes the next level's node list.
// Rows are regrouped only every SECOND level (see k_route), so the node list alternates between
//   * even levels: nodes own contiguous row ranges [start, start+len) of the level's buffer;
//   * odd levels: nodes are the two halves of their parent's range (start/len = the parent's, `dir`
//     = 0 left / 1 right); k_hist_build filters the parent's rows by the parent's decision.
// Even depth (next level odd): next ranges = parent ranges, tile prefix built here; node_nl is zeroed
//   for the filtered histogram pass to count left-goers into.
// Odd depth (next level even): the children's ranges are only known after k_route, which fills each
//   odd node's region of the next buffer from both ends; this kernel sets up those cursors
//   (curs[c] = {front, back, region start, region end}, from the parent's left count prev_nl) and
// the fields of a decision the plan reads (the 176-B record carries a 1024-bit set it never needs)
struct DecLite { int feat; double wl, wr; };
__device__ __forceinline__ DecLite dec_lite(const Dec* d) { return DecLite{d->feat, d->wl, d->wr}; }

//   k_ranges turns the final cursors into ranges + tile prefix.

__device__ __forceinline__ int wave_excl_scan(int v, int* total) {
  const int lane = threadIdx.x & 63;
  int x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  *total = __shfl(x, 63, 64);
  return x - v;
}

// The plan of a level of <= 64 nodes on ONE wave, lane = node, every prefix a wave scan in registers: the same
// numbering, children and tile prefixes as the block version below (whose four block scans each cost three
// barriers and a serial pass over the waves). The next level's tile prefix is computed from the children each
// lane creates (its children are consecutive in the next list), so the next list is never read back.
__device__ void plan_wave(
    const Node* __restrict__ nodes, int n, Dec* __restrict__ dec, int* __restrict__ node_nl,
    const int* __restrict__ prev_nl, int4* __restrict__ curs, int* __restrict__ child_l, int* __restrict__ child_r,
    Node* __restrict__ next, int* __restrict__ next_tile_prefix, int* __restrict__ next_meta,
    int* __restrict__ next_build_prefix, int* __restrict__ counters, int depth, int max_depth, double min_w,
    int cap_next, int leaf_cap) {
  const int i = threadIdx.x;                       // lane = node
  const bool odd = depth & 1;
  const bool live = i < n;
  Node nd{0, 0, 0, -1, -1, 0, 0, 0};
  DecLite d{-1, 0.0, 0.0};
  if (live) {
    nd = nodes[i];
    d = dec_lite(dec + i);
    if (!odd) {
      node_nl[i] = 0;
    } else {
      const int nl = nd.parent >= 0 ? prev_nl[nd.parent] : 0;
      const int cs = nd.start + (nd.dir ? nl : 0);
      const int ce = nd.dir ? nd.start + nd.len : nd.start + nl;
      curs[i] = make_int4(cs, ce, cs, ce);
    }
  }
  const bool split = live && d.feat >= 0;
  const bool la = split && depth + 1 < max_depth && d.wl >= 2.0 * min_w;
  const bool ra = split && depth + 1 < max_depth && d.wr >= 2.0 * min_w;
  int act_total;
  const int act_off = wave_excl_scan((la ? 1 : 0) + (ra ? 1 : 0), &act_total);
  int ao = act_off;
  int li = -1, ri = -1;
  if (la) { if (ao < cap_next) li = ao; ++ao; }
  if (ra) { if (ao < cap_next) ri = ao; ++ao; }
  const int lv = !live ? 0 : (!split ? 1 : 2 - (li >= 0) - (ri >= 0));
  const int leaf_base0 = counters[0];
  int n_leaves_new;
  int lo = leaf_base0 + wave_excl_scan(lv, &n_leaves_new);
  if (live) {
    if (!split) {
      const int lid = min(lo, leaf_cap - 1);
      child_l[i] = -1 - lid; child_r[i] = -1 - lid;
    } else {
      child_l[i] = li >= 0 ? li : -1 - min(lo++, leaf_cap - 1);
      child_r[i] = ri >= 0 ? ri : -1 - min(lo++, leaf_cap - 1);
      if (li >= 0 && ri >= 0) {
        const bool build_left = d.wl <= d.wr;
        next[li] = Node{nd.start, nd.len, build_left ? 1 : 0, i, ri, 0, 0, 0};
        next[ri] = Node{nd.start, nd.len, build_left ? 0 : 1, i, li, 1, 0, 0};
      } else if (li >= 0) {
        next[li] = Node{nd.start, nd.len, 1, i, -1, 0, 0, 0};
      } else if (ri >= 0) {
        next[ri] = Node{nd.start, nd.len, 1, i, -1, 1, 0, 0};
      }
    }
  }
  const int nn = min(act_total, cap_next);
  if (i == 0) counters[0] = min(leaf_base0 + n_leaves_new, leaf_cap);
  if (odd) {
    if (i == 0) { next_meta[0] = nn; next_meta[1] = 0; next_meta[2] = 0; }
    return;
  }
  // even depth: the next (odd) level's nodes keep the parent's range — tiles of its children, in child order
  const int kt = (nd.len + TILE - 1) / TILE;
  const bool lb = li >= 0 && (ri < 0 || d.wl <= d.wr);
  const bool rb = ri >= 0 && !(li >= 0 && d.wl <= d.wr);
  int tot, totb;
  int off = wave_excl_scan((li >= 0 ? kt : 0) + (ri >= 0 ? kt : 0), &tot);
  int offb = wave_excl_scan((lb ? kt : 0) + (rb ? kt : 0), &totb);
  if (li >= 0) { next_tile_prefix[li] = off; next_build_prefix[li] = offb; off += kt; offb += lb ? kt : 0; }
  if (ri >= 0) { next_tile_prefix[ri] = off; next_build_prefix[ri] = offb; }
  if (i == 0) {
    next_tile_prefix[nn] = tot; next_build_prefix[nn] = totb;
    next_meta[0] = nn; next_meta[1] = tot; next_meta[2] = totb;
  }
}

__device__ void plan_body(
    const Node* __restrict__ nodes, const int* __restrict__ meta, Dec* __restrict__ dec,
    int* __restrict__ node_nl, const int* __restrict__ prev_nl, int4* __restrict__ curs,
    int* __restrict__ child_l, int* __restrict__ child_r,
    Node* __restrict__ next, int* __restrict__ next_tile_prefix, int* __restrict__ next_meta,
    int* __restrict__ next_build_prefix,
    int* __restrict__ counters, int* __restrict__ scratch /* >= cap_cur ints */,
    int depth, int max_depth, double min_w, int cap_next, int leaf_cap, PlanReduce pr) {
  __shared__ int sh[17];
  const int n = meta[0];
  const int T = blockDim.x, tid = threadIdx.x;
  if (pr.cand) {
    for (int node = tid >> 6; node < n; node += T >> 6)
      reduce_node(pr.cand, node, pr.F, pr.feat_ok, pr.k_cols, pr.seed, depth, dec, pr.node_ok, pr.fgroup, tid & 63,
                  pr.cfs, pr.ccap);
    __syncthreads();                     // the block's own decisions (global) before the plan reads them
  }
  if (n <= 64 && !pr.no_wave) {       // small level: wave 0 alone (the other waves are done)
    if (tid < 64)
      plan_wave(nodes, n, dec, node_nl, prev_nl, curs, child_l, child_r, next, next_tile_prefix, next_meta,
                next_build_prefix, counters, depth, max_depth, min_w, cap_next, leaf_cap);
    return;
  }
  const bool odd = depth & 1;
  int total;
  const int perN = (n + T - 1) / T;
  const int na = min(n, tid * perN), nb2 = min(n, na + perN);
  // per-node bookkeeping of the CURRENT level
  for (int i = na; i < nb2; ++i) {
    const Node nd = nodes[i];
    if (!odd) {
      node_nl[i] = 0;
    } else {
      const int nl = nd.parent >= 0 ? prev_nl[nd.parent] : 0;
      const int cs = nd.start + (nd.dir ? nl : 0);
      const int ce = nd.dir ? nd.start + nd.len : nd.start + nl;
      curs[i] = make_int4(cs, ce, cs, ce);
    }
  }
  // 1. children: active / leaf classification, compaction with capacity
  int act_cnt = 0;
  for (int i = na; i < nb2; ++i) {
    const DecLite d = dec_lite(dec + i);
    int a = 0;
    if (d.feat >= 0 && depth + 1 < max_depth) {
      // child activity is decided from GLOBAL (all-reduced) weights so every rank plans alike
      a += (d.wl >= 2.0 * min_w) ? 1 : 0;
      a += (d.wr >= 2.0 * min_w) ? 1 : 0;
    }
    act_cnt += a;
  }
  int act_off = block_excl_scan(act_cnt, sh, &total);
  // recount leaves given capacity overflow, store flags in scratch[i] (bit0 left active, bit1 right active)
  int leaf_cnt = 0;
  {
    int ao = act_off;
    for (int i = na; i < nb2; ++i) {
      const DecLite d = dec_lite(dec + i);
      int flags = 0, lv = 0;
      if (d.feat < 0) { lv = 1; }
      else {
        const bool la = depth + 1 < max_depth && d.wl >= 2.0 * min_w;
        const bool ra = depth + 1 < max_depth && d.wr >= 2.0 * min_w;
        if (la) { if (ao < cap_next) flags |= 1; ++ao; }
        if (ra) { if (ao < cap_next) flags |= 2; ++ao; }
        lv = 2 - ((flags & 1) + ((flags >> 1) & 1));
      }
      scratch[i] = flags;
      leaf_cnt += lv;
    }
  }
  const int leaf_base0 = counters[0];
  __syncthreads();
  int leaf_off = block_excl_scan(leaf_cnt, sh, &total);
  const int n_leaves_new = total;
  int ao = act_off;
  int lo = leaf_base0 + leaf_off;
  for (int i = na; i < nb2; ++i) {
    const DecLite d = dec_lite(dec + i);
    const Node nd = nodes[i];
    const int flags = scratch[i];
    if (d.feat < 0) {
      const int lid = min(lo++, leaf_cap - 1);
      child_l[i] = -1 - lid; child_r[i] = -1 - lid;
      continue;
    }
    const bool la = depth + 1 < max_depth && d.wl >= 2.0 * min_w;
    const bool ra = depth + 1 < max_depth && d.wr >= 2.0 * min_w;
    int li = -1, ri = -1;
    if (la) { if (flags & 1) li = ao; ++ao; }
    if (ra) { if (flags & 2) ri = ao; ++ao; }
    child_l[i] = (li >= 0) ? li : -1 - min(lo++, leaf_cap - 1);
    child_r[i] = (ri >= 0) ? ri : -1 - min(lo++, leaf_cap - 1);
    // children of an even node inherit its range (odd level); children of an odd node get theirs in k_ranges
    if (li >= 0 && ri >= 0) {
      const bool build_left = d.wl <= d.wr;  // global weights: identical choice on every rank
      next[li] = Node{nd.start, nd.len, build_left ? 1 : 0, i, ri, 0, 0, 0};
      next[ri] = Node{nd.start, nd.len, build_left ? 0 : 1, i, li, 1, 0, 0};
    } else if (li >= 0) {
      next[li] = Node{nd.start, nd.len, 1, i, -1, 0, 0, 0};
    } else if (ri >= 0) {
      next[ri] = Node{nd.start, nd.len, 1, i, -1, 1, 0, 0};
    }
  }
  __syncthreads();
  __shared__ int s_nnext;
  if (tid == T - 1) s_nnext = min(act_off + act_cnt, cap_next);  // only the last thread holds the total
  __syncthreads();
  const int nn = s_nnext;
  if (tid == 0) counters[0] = min(leaf_base0 + n_leaves_new, leaf_cap);
  if (!odd) {
    level_tile_prefix(next, nn, next_tile_prefix, next_build_prefix, next_meta, sh);
  } else if (tid == 0) {
    next_meta[0] = nn; next_meta[1] = 0; next_meta[2] = 0;
  }
}

__global__ __launch_bounds__(1024) void k_plan(
    const Node* __restrict__ nodes, const int* __restrict__ meta, Dec* __restrict__ dec,
    int* __restrict__ node_nl, const int* __restrict__ prev_nl, int4* __restrict__ curs,
    int* __restrict__ child_l, int* __restrict__ child_r,
    Node* __restrict__ next, int* __restrict__ next_tile_prefix, int* __restrict__ next_meta,
    int* __restrict__ next_build_prefix, int* __restrict__ counters, int* __restrict__ scratch,
    int depth, int max_depth, double min_w, int cap_next, int leaf_cap, PlanReduce pr) {
  plan_body(nodes, meta, dec, node_nl, prev_nl, curs, child_l, child_r, next, next_tile_prefix, next_meta,
            next_build_prefix, counters, scratch, depth, max_depth, min_w, cap_next, leaf_cap, pr);
}

template <bool GRP>
__global__ __launch_bounds__(256) void k_split_find(
    double* __restrict__ hist, int slot_doubles, const int* __restrict__ meta, int F,
    const int* __restrict__ nbins_f, const int* __restrict__ iscat_f, const int* __restrict__ mono_f,
    SplitParams p, int level, Cand* __restrict__ cand, double* __restrict__ root_w,
    const float* __restrict__ edges, int adapt_nb, int f0, int FL, Derive dv) {
  split_find_body<GRP>(hist, slot_doubles, meta, F, nbins_f, iscat_f, mono_f, p, level, cand, root_w, edges, adapt_nb,
                       f0, FL, dv);
}

// k_split_find with the level's k_plan folded into its LAST block (single process, <= PLAN_REDUCE_MAX nodes): every
// (node, feature) block publishes its candidate with an agent-scope RELEASE ticket on `done`; the block drawing the
// final ticket acquires (L2 invalidate) and runs the plan — reduce_node over the candidates, child numbering, the
// next level's node list and tile prefixes — with its 256 threads. One launch per level instead of two.
struct PlanArgs {
  const Node* nodes;
  const int* meta;
  Dec* dec;
  int* node_nl;
  const int* prev_nl;
  int4* curs;
  int* child_l;
  int* child_r;
  Node* next;
  int* next_tp;
  int* next_meta;
  int* next_bp;
  int* counters;
  int* scratch;
  int depth, max_depth, cap_next, leaf_cap;
  double min_w;
  PlanReduce pr;
  int* done;       // zero before the launch; the last block resets it
};

__global__ __launch_bounds__(256) void k_split_find_plan(
    double* __restrict__ hist, int slot_doubles, const int* __restrict__ meta, int F,
    const int* __restrict__ nbins_f, const int* __restrict__ iscat_f, const int* __restrict__ mono_f,
    SplitParams p, int level, Cand* __restrict__ cand, double* __restrict__ root_w,
    const float* __restrict__ edges, int adapt_nb, int f0, int FL, Derive dv, PlanArgs pa) {
  split_find_body<false>(hist, slot_doubles, meta, F, nbins_f, iscat_f, mono_f, p, level, cand, root_w, edges,
                         adapt_nb, f0, FL, dv);
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int total = (int)(gridDim.x * gridDim.y);
    s_last = __hip_atomic_fetch_add(pa.done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT) == total - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  plan_body(pa.nodes, pa.meta, pa.dec, pa.node_nl, pa.prev_nl, pa.curs, pa.child_l, pa.child_r, pa.next, pa.next_tp,
            pa.next_meta, pa.next_bp, pa.counters, pa.scratch, pa.depth, pa.max_depth, pa.min_w, pa.cap_next,
            pa.leaf_cap, pa.pr);
  if (threadIdx.x == 0) __hip_atomic_store(pa.done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Interaction constraints (GlobalInteractionConstraints / BranchInteractionConstraints): a child may split
// on the features its parent allowed AND that interact with the parent's split feature:
// ok[child][f] = ok[parent][f] & map[parent split feature][f]. grid = next-level capacity, block 64.
__global__ __launch_bounds__(64) void k_ic_next(const Node* __restrict__ next, const int* __restrict__ next_meta,
                                                const Dec* __restrict__ dec, const unsigned char* __restrict__ ok_cur,
                                                const unsigned char* __restrict__ ic_map, int F,
                                                unsigned char* __restrict__ ok_next) {
  const int c = blockIdx.x;
  if (c >= next_meta[0]) return;
  const int par = next[c].parent;
  const int sf = dec[par].feat;
  for (int f = threadIdx.x; f < F; f += 64)
    ok_next[(size_t)c * F + f] = (sf >= 0 && ok_cur[(size_t)par * F + f] && ic_map[(size_t)sf * F + f]) ? 1 : 0;
}

// k_ranges: after k_route filled the odd level's regions, give each even-level node its range
// (left child: [region start, front); right child: [back, region end)) and build the tile prefix.
__global__ __launch_bounds__(1024) void k_ranges(Node* __restrict__ next, const int4* __restrict__ curs,
                                                 int* __restrict__ tp, int* __restrict__ bp, int* __restrict__ meta) {
  __shared__ int sh[17];
  const int nn = meta[0];
  for (int i = threadIdx.x; i < nn; i += blockDim.x) {
    Node nd = next[i];
    const int4 c = curs[nd.parent];
    if (nd.dir == 0) { nd.start = c.z; nd.len = c.x - c.z; }
    else { nd.start = c.y; nd.len = c.w - c.y; }
    next[i] = nd;
  }
  __syncthreads();
  level_tile_prefix(next, nn, tp, bp, meta, sh);
}

// k_zero_hist: zero the compact build slots (slot = parent) of next-level nodes built directly.
__global__ void k_zero_hist(double* __restrict__ hbuild, const Node* __restrict__ next,
                            const int* __restrict__ meta, int slot_doubles) {
  const int node = blockIdx.y;
  if (node >= meta[0] || !next[node].build) return;
  double* s = hbuild + (size_t)next[node].parent * slot_doubles;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < slot_doubles; i += gridDim.x * blockDim.x) s[i] = 0.0;
}

// k_hist_pack: feature-sliced reduce-scatter staging. Node slots [n][slot] (bin-major (bin, f) pairs, then
// naYY[F], wYY) -> dst[W][n][E] where rank r's chunk holds, per node, the same layout restricted to its
// features [r*Fs, r*Fs + Fs): (bin, f') pairs, naYY[f'], wYY (E = Fs*2*NBIN + Fs + 1). Features past F
// are zero-filled. After reduce_scatter each rank owns the GLOBAL histograms of its slice, in the layout
// k_split_find reads with F = Fs.
template <typename TO>
__global__ void k_hist_pack(const double* __restrict__ src, int slot, int F, int Fs, int W, int n,
                            TO* __restrict__ dst) {
  const long long E = (long long)Fs * 2 * NBIN + Fs + 1;
  const long long total = (long long)W * n * E;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long e = i % E;
    const long long rn = i / E;
    const int node = (int)(rn % n), r = (int)(rn / n);
    const double* sl = src + (size_t)node * slot;
    double v;
    if (e < (long long)Fs * 2 * NBIN) {
      const int bin = (int)(e / (2 * Fs)), rem = (int)(e % (2 * Fs));
      const int f = r * Fs + (rem >> 1);
      v = f < F ? sl[(size_t)bin * 2 * F + 2 * f + (rem & 1)] : 0.0;
    } else if (e < (long long)Fs * 2 * NBIN + Fs) {
      const int f = r * Fs + (int)(e - (long long)Fs * 2 * NBIN);
      v = f < F ? sl[(size_t)F * 2 * NBIN + f] : 0.0;
    } else {
      v = sl[(size_t)F * 2 * NBIN + F];
    }
    dst[i] = (TO)v;
  }
}

// ------------------------------------------------------------------------------------------------
// k_route: regroups the rows of an EVEN level e two levels down at once. Rows are physically moved only
// every second level: level e+1 is histogrammed by filtering the level-e ranges (k_hist_build<true>), so a
// depth-6 tree moves its rows twice instead of five times and needs no separate counting pass.
//   block = one TILE (2048 rows) of a level-e node; 8 waves x 256 rows, lane = row (4 rows per lane).
//   Each row gets a slot q = 2*dirA + dirB (its grandchild); rows of a continuing grandchild move into
//   the region of their level-(e+1) node: left grandchildren fill it from the front, right ones from the
//   back (one atomic per (tile, slot) on curs). Rows that reach a leaf on the way are simply not moved:
//   leaf ids and leaf sums come from k_leaf_assign over the ORIGINAL row order after the last level, so the
//   row payload is only the bins and the histogram inputs (wY, and w for weighted rows) — no row index.
// Order inside a region is not preserved: histograms are fixed-point integer sums (order independent)
// and nothing else depends on the row order within a node.
#define LW 8              // waves per route block (MEASURED: 4 waves x 8 rows per lane 169 -> 182 us)
#define LROWS (TILE / LW) // rows per wave (256)
#define LU (LROWS / 64)   // rows per lane (4)
#define LMAXW 16          // max words (64 features) kept in registers per row on the fast path

// NV > 0 (rows of NV x 16 B): each row is loaded ONCE into registers up front, split bytes are picked from
// those registers and the move stores them back (one HBM read per row).
__device__ __forceinline__ unsigned pick_word(uint4 v, int wi) {
  // a compare/select chain on values (no runtime-indexed register array -> no scratch)
  unsigned r = v.x;
  r = wi == 1 ? v.y : r;
  r = wi == 2 ? v.z : r;
  r = wi == 3 ? v.w : r;
  return r;
}
__device__ __forceinline__ int row_byte(uint4 v0, uint4 v1, int f) {
  const int wi = f >> 2;
  const unsigned w = wi < 4 ? pick_word(v0, wi) : pick_word(v1, wi - 4);
  return (w >> (8 * (f & 3))) & 0xFF;
}
__device__ __forceinline__ int row_byte4(uint4 v0, uint4 v1, uint4 v2, uint4 v3, int f) {
  return f < 32 ? row_byte(v0, v1, f) : row_byte(v2, v3, f - 32);
}
// the aligned row word holding column f (f % 4 == 0: a wide-categorical group)
__device__ __forceinline__ unsigned row_word(uint4 v0, uint4 v1, int f) {
  const int wi = f >> 2;
  return wi < 4 ? pick_word(v0, wi) : pick_word(v1, wi - 4);
}
__device__ __forceinline__ unsigned row_word4(uint4 v0, uint4 v1, uint4 v2, uint4 v3, int f) {
  return f < 32 ? row_word(v0, v1, f) : row_word(v2, v3, f - 32);
}
// a decision's row key from registers (NV > 0) or memory: the split byte, or a group split's row word
// (GRP: the tree can hold group splits; without groups the route / leaf walk compile to the byte path only)
template <int NV, bool GRP>
__device__ __forceinline__ unsigned split_key(bool grp, int f, uint4 v0, uint4 v1, uint4 v2, uint4 v3,
                                              const uint8_t* __restrict__ bins, long long row, int stride, long long N,
                                              int planar) {
  if (GRP && grp) {
    if (NV > 0 && f < NV * 16) return NV > 2 ? row_word4(v0, v1, v2, v3, f) : row_word(v0, v1, f);
    return *reinterpret_cast<const unsigned*>(bins + bin_off(row, f, stride, N, planar));
  }
  return (NV > 0 && f >= NV * 16) ? bins[bin_off(row, f, stride, N, planar)]
         : NV > 2 ? (unsigned)row_byte4(v0, v1, v2, v3, f) : NV > 0 ? (unsigned)row_byte(v0, v1, f)
                  : bins[bin_off(row, f, stride, N, planar)];
}

template <int NV, bool GRP>
__device__ __forceinline__ void route_tile(
    const uint8_t* __restrict__ sbins, const float* __restrict__ say, const float* __restrict__ saw,
    uint8_t* __restrict__ dbins, float* __restrict__ day, float* __restrict__ daw, int stride,
    const Node* __restrict__ nodesA, const int* __restrict__ tpA, const int* __restrict__ metaA,
    const Dec* __restrict__ decA, const int* __restrict__ clA, const int* __restrict__ crA,
    const Dec* __restrict__ decB, const int* __restrict__ clB, const int* __restrict__ crB,
    int4* __restrict__ curs, long long N, int planar, uint8_t* __restrict__ lvl2,
    const uint8_t* __restrict__ fdir, int t) {
  const int n_nodes = metaA[0];
  __shared__ Dec sA, sB[2];
  __shared__ int sC[2], sG[4], sBase[4], sL[4];
  __shared__ int sCnt[LW][4];
  const int node = find_node(tpA, n_nodes, t);
  const Node nd = nodesA[node];
  const int tin = t - tpA[node];
  const int r0 = nd.start + tin * TILE;
  const int r1 = min(r0 + TILE, nd.start + nd.len);
  constexpr int NI = (int)(sizeof(Dec) / 4);
  if (threadIdx.x < NI) ((int*)&sA)[threadIdx.x] = ((const int*)(decA + node))[threadIdx.x];
  if (threadIdx.x < 2) sC[threadIdx.x] = threadIdx.x == 0 ? clA[node] : crA[node];
  __syncthreads();
  if (threadIdx.x < 4) {
    // slot q -> continuing grandchild (>= 0), else the row stops at a leaf
    const int q = threadIdx.x, c = sC[q >> 1];
    sG[q] = c < 0 ? -1 : ((q & 1) ? crB[c] : clB[c]);
    // lvl2 code of slot q: the grandchild's node index, or 128 + the leaf the row stops at
    const int g = c < 0 ? c : sG[q];
    sL[q] = g >= 0 ? g : 128 + (-1 - g);
  }
  for (int k = 0; k < 2; ++k) {
    const int c = sC[k];
    if (c >= 0 && threadIdx.x < NI) ((int*)&sB[k])[threadIdx.x] = ((const int*)(decB + c))[threadIdx.x];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int featA = sA.feat;
  // per-tile constants of the two decision levels (wide-categorical group splits read a row word)
  const bool grpA = sA.is_cat == GROUP_CAT;
  const int fB0 = sC[0] >= 0 ? sB[0].feat : -1, fB1 = sC[1] >= 0 ? sB[1].feat : -1;
  const bool grpB0 = sC[0] >= 0 && sB[0].is_cat == GROUP_CAT, grpB1 = sC[1] >= 0 && sB[1].is_cat == GROUP_CAT;
  const int wbase = r0 + wid * LROWS;
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int q[LU], rank[LU];
  bool mv[LU];
  int cnt[4] = {0, 0, 0, 0};
  uint4 rv0[LU], rv1[LU], rv2[LU], rv3[LU];
  float ry[LU], rw[LU];
#pragma unroll
  for (int u = 0; u < LU; ++u) {
    const int row = min(wbase + u * 64 + lane, r1 - 1);   // clamped into the node: no divergence
    if (NV > 0) {
      // planar (NV == 4): words 0-7 from plane 0, 8-15 from plane 1 — the same registers as a 64-B row
      const uint4* s4 = (const uint4*)(sbins + (planar ? (size_t)row * 32 : (size_t)row * stride));
      const uint4* s4b = planar ? (const uint4*)(sbins + ((size_t)N + row) * 32) : s4 + 2;
      rv0[u] = s4[0];
      rv1[u] = NV > 1 ? s4[1] : make_uint4(0u, 0u, 0u, 0u);
      rv2[u] = NV > 2 ? s4b[0] : make_uint4(0u, 0u, 0u, 0u);
      rv3[u] = NV > 3 ? s4b[1] : make_uint4(0u, 0u, 0u, 0u);
    }
    ry[u] = say[row];
    rw[u] = saw ? saw[row] : 1.f;
  }
#pragma unroll
  for (int u = 0; u < LU; ++u) {
    const int row = wbase + u * 64 + lane;
    const bool valid = row < r1;
    int dA = 0, dB = 0;
    // (a split column past the registers — narrow copies, lp > 0 — is read from the source)
    if (fdir) {
      dA = valid && featA >= 0 ? fdir[row] : 0;
    } else if (valid && featA >= 0)
      dA = dec_go_left_key<GRP>(&sA, split_key<NV, GRP>(grpA, featA, rv0[u], rv1[u], rv2[u], rv3[u], sbins, row, stride,
                                                        N, planar)) ? 0 : 1;
    if (valid && sC[dA] >= 0) {
      const Dec* b = &sB[dA];
      const int fb = dA ? fB1 : fB0;
      if (fb >= 0)
        dB = dec_go_left_key<GRP>(b, split_key<NV, GRP>(dA ? grpB1 : grpB0, fb, rv0[u], rv1[u], rv2[u], rv3[u], sbins,
                                                        row, stride, N, planar)) ? 0 : 1;
    }
    q[u] = 2 * dA + dB;
    mv[u] = valid && sG[q[u]] >= 0;
    if (lvl2 && valid) lvl2[row] = (uint8_t)sL[q[u]];   // (e = 0: rows in original order)
    rank[u] = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool mine = mv[u] && q[u] == k;
      const unsigned long long bm = __ballot(mine);
      if (mine) rank[u] = cnt[k] + __popcll(bm & below);
      cnt[k] += __popcll(bm);
    }
  }
  if (lane == 0) for (int k = 0; k < 4; ++k) sCnt[wid][k] = cnt[k];
  __syncthreads();
  if (threadIdx.x < 4) {
    const int k = threadIdx.x;
    int tot = 0;
    for (int w = 0; w < LW; ++w) tot += sCnt[w][k];
    int base = 0;
    if (tot > 0) {
      int4* cu = curs + sC[k >> 1];
      base = (k & 1) ? atomicSub(&cu->y, tot) - tot : atomicAdd(&cu->x, tot);
    }
    sBase[k] = base;
  }
  __syncthreads();
  int off[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    off[k] = sBase[k];
    for (int w = 0; w < wid; ++w) off[k] += sCnt[w][k];
  }
  const int W = stride >> 2;
  const unsigned* sb32 = (const unsigned*)sbins;
  unsigned* db32 = (unsigned*)dbins;
#pragma unroll
  for (int u = 0; u < LU; ++u) {
    if (!mv[u]) continue;
    const int row = wbase + u * 64 + lane;
    int pos = rank[u];
#pragma unroll
    for (int k = 0; k < 4; ++k) if (q[u] == k) pos += off[k];
    unsigned* dst = db32 + (size_t)pos * (planar ? 8 : W);
    if (NV > 0) {
      uint4* d4 = (uint4*)dst;
      uint4* d4b = planar ? (uint4*)(db32 + ((size_t)N + pos) * 8) : d4 + 2;
      d4[0] = rv0[u];
      if (NV > 1) d4[1] = rv1[u];
      if (NV > 2) d4b[0] = rv2[u];
      if (NV > 3) d4b[1] = rv3[u];
    } else if (planar) {
      for (int pl = 0; pl < (W >> 3); ++pl) {
        const unsigned* src = sb32 + ((size_t)pl * N + row) * 8;
        unsigned* d = db32 + ((size_t)pl * N + pos) * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) d[k] = src[k];
      }
    } else {
      const unsigned* src = sb32 + (size_t)row * W;
      if (W <= LMAXW) {
        unsigned v[LMAXW];
#pragma unroll
        for (int k = 0; k < LMAXW; ++k) if (k < W) v[k] = src[k];
#pragma unroll
        for (int k = 0; k < LMAXW; ++k) if (k < W) dst[k] = v[k];
      } else {
        for (int k = 0; k < W; ++k) dst[k] = src[k];
      }
    }
    day[pos] = ry[u];
    if (daw) daw[pos] = rw[u];
  }
}

// k_ranges work folded into the route's LAST block (ro.done != null): every block counts itself out on ro.done
// after its cursor atomics have returned (it used their results), so the block that draws the final ticket sees the
// final cursors. The cursors are read back with agent-scope atomic loads (they were only ever updated by atomics at
// the coherence point; no fence / L2 write-back is needed), the node list and prefixes are written with plain
// stores that the next kernel reads. Saves one launch per route (MEASURED r5: k_ranges 4.6 us, 2 per tree).
struct RangesOut {
  Node* next;
  int* tp;
  int* bp;
  int* meta;
  int* done;     // zero before the launch; the last block resets it
};
template <int NV, bool GRP>
__global__ __launch_bounds__(LW * 64) void k_route(
    const uint8_t* __restrict__ sbins, const float* __restrict__ say, const float* __restrict__ saw,
    uint8_t* __restrict__ dbins, float* __restrict__ day, float* __restrict__ daw, int stride,
    const Node* __restrict__ nodesA, const int* __restrict__ tpA, const int* __restrict__ metaA,
    const Dec* __restrict__ decA, const int* __restrict__ clA, const int* __restrict__ crA,
    const Dec* __restrict__ decB, const int* __restrict__ clB, const int* __restrict__ crB,
    int4* __restrict__ curs, long long N, int planar, uint8_t* __restrict__ lvl2,
    const uint8_t* __restrict__ fdir /*root route: per row the root split's direction (k_row_dir), or null*/,
    RangesOut ro) {
  const int t = blockIdx.x;
  if (t < metaA[1])
    route_tile<NV, GRP>(sbins, say, saw, dbins, day, daw, stride, nodesA, tpA, metaA, decA, clA, crA, decB, clB, crB,
                        curs, N, planar, lvl2, fdir, t);
  if (!ro.done) return;
  __shared__ int s_last;
  __shared__ int sh[17];
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(ro.done, 1) == (int)gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  const int nn = ro.meta[0];
  for (int i = threadIdx.x; i < nn; i += blockDim.x) {
    Node nd = ro.next[i];
    int* cp = (int*)(curs + nd.parent);
    if (nd.dir == 0) {
      const int z = __hip_atomic_load(cp + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      nd.start = z;
      nd.len = __hip_atomic_load(cp + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - z;
    } else {
      const int y = __hip_atomic_load(cp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      nd.start = y;
      nd.len = __hip_atomic_load(cp + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - y;
    }
    ro.next[i] = nd;
  }
  __syncthreads();
  level_tile_prefix(ro.next, nn, ro.tp, ro.bp, ro.meta, sh);
  if (threadIdx.x == 0) atomicExch(ro.done, 0);
}

// ------------------------------------------------------------------------------------------------
// k_row_dir: every row's side of the root split (0 left, 1 right), one byte per row in the original order. Narrow
// runs read the root split's column from a plane nothing else of level 1 reads: the two level-1 histogram blocks
// and the root route then read these bytes (1 B per row) instead of that plane (32 B per row each).
__global__ __launch_bounds__(256) void k_row_dir(const uint8_t* __restrict__ bins, int stride, long long N, int planar,
                                                 const Dec* __restrict__ dec, uint8_t* __restrict__ out) {
  __shared__ Dec sd;
  if (threadIdx.x < (int)(sizeof(Dec) / 4)) ((int*)&sd)[threadIdx.x] = ((const int*)dec)[threadIdx.x];
  __syncthreads();
  const int f = sd.feat;
  for (long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x; row < N; row += (long long)gridDim.x * blockDim.x)
    out[row] = (f >= 0 && !dec_go_left_key(&sd, sd.is_cat == GROUP_CAT
                                                   ? *reinterpret_cast<const unsigned*>(bins + bin_off(row, f, stride, N, planar))
                                                   : (unsigned)bins[bin_off(row, f, stride, N, planar)])) ? 1 : 0;
}

// ------------------------------------------------------------------------------------------------
// k_leaf_assign: after the last level, every row walks the tree from the root in ORIGINAL row order
// (master bins, coalesced) to its leaf: leaf_of_row[row] and the per-leaf Newton sums (gamma numerator /
// denominator planes) as int64 fixed point (scales from k_qscale; sums are exact and order independent ->
// deterministic). GBM.java fitBestConstants / AddTreeContributions consume these sums.
// The tree is staged in LDS as 16-B {feat, bin | na_left << 16 | is_cat << 17, child_l, child_r} records
// (flattened by level), so a row's walk is D dependent LDS reads instead of D chains of dependent global
// loads (MEASURED on the global walk: 419 us per tree at 11M rows, latency-bound). Categorical bitsets stay
// in the global Dec records (read only on categorical splits). Small leaf sets are privatised in LDS.
// Dynamic LDS: [2*leaf_cap u64 sums (if leaf_cap <= LEAF_LDS_MAX)] [n_nodes int4 (if <= LEAF_TREE_MAX)].
#define LEAF_LDS_MAX 2048
#define LEAF_TREE_MAX 2048
struct LevelPtrs { const Dec* dec; const int* cl; const int* cr; long long cap; };

template <int NV, bool GRP>
__device__ __forceinline__ void leaf_assign_body(
    const uint8_t* __restrict__ bins, int stride, long long N, const LevelPtrs* __restrict__ lv, int D,
    const float* __restrict__ an, const float* __restrict__ ad, const double* __restrict__ qs,
    int* __restrict__ leaf_of_row, unsigned long long* __restrict__ leafq, int leaf_cap, int n_nodes, int planar,
    const uint8_t* __restrict__ lvl2 /*null, or every row's level-2 node / 128 + leaf (k_route of the root)*/) {
  extern __shared__ __align__(16) unsigned char la_smem[];
  __shared__ int sbase[TP_MAXL_DEV + 1];
  const bool lds = leaf_cap <= LEAF_LDS_MAX;
  const bool tl = n_nodes <= LEAF_TREE_MAX;
  unsigned long long* sq = (unsigned long long*)la_smem;
  int4* st = (int4*)(la_smem + (lds ? (size_t)16 * leaf_cap : 0));
  if (threadIdx.x == 0) {
    int b = 0;
    for (int d = 0; d < D; ++d) { sbase[d] = b; b += (int)lv[d].cap; }
    sbase[D] = b;
  }
  if (lds)
    for (int i = threadIdx.x; i < 2 * leaf_cap; i += blockDim.x) sq[i] = 0ull;
  __syncthreads();
  if (tl) {
    for (int d = 0; d < D; ++d) {
      const int c = (int)lv[d].cap, b = sbase[d];
      for (int i = threadIdx.x; i < c; i += blockDim.x) {
        const Dec* dc = lv[d].dec + i;
        st[b + i] = make_int4(dc->feat, (dc->bin & 0xFFFF) | ((dc->na_left != 0) << 16) | ((dc->is_cat != 0) << 17) |
                                            ((dc->is_cat == GROUP_CAT) << 18),
                              lv[d].cl[i], lv[d].cr[i]);
      }
    }
  }
  __syncthreads();
  const float sn = (float)qs[6], sd = (float)qs[7];
  for (long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x; row < N;
       row += (long long)gridDim.x * blockDim.x) {
    uint4 v0 = make_uint4(0u, 0u, 0u, 0u), v1 = v0, v2 = v0, v3 = v0;
    if (NV > 0) {
      const uint4* s4 = (const uint4*)(bins + (planar ? (size_t)row * 32 : (size_t)row * stride));
      const uint4* s4b = planar ? (const uint4*)(bins + ((size_t)N + row) * 32) : s4 + 2;
      v0 = s4[0];
      if (NV > 1) v1 = s4[1];
      if (NV > 2) v2 = s4b[0];
      if (NV > 3) v3 = s4b[1];
    }
    const float a_n = an[row], a_d = ad[row];    // issued before the walk: latency overlaps it
    int i = 0, leaf = 0, d0 = 0;
    if (lvl2) {                                  // the root route's level-2 position: walk from level 2
      const int code = lvl2[row];
      d0 = (code & 128) ? D : 2;
      if (code & 128) leaf = code & 127; else i = code;
    }
    for (int d = d0; d < D; ++d) {
      int c;
      if (tl) {
        const int4 e = st[sbase[d] + i];
        if (e.x < 0) {
          c = e.z;                               // terminal node: child_l == child_r == its leaf
        } else if (GRP && ((e.y >> 18) & 1)) {   // wide-categorical group: the row word, the record in global
          const Dec* dc = lv[d].dec + i;
          c = dec_go_left_key<GRP>(dc, split_key<NV, GRP>(true, e.x, v0, v1, v2, v3, bins, row, stride, N, planar))
                  ? e.z : e.w;
        } else {
          const int b = (NV > 0 && e.x >= NV * 16) ? bins[bin_off(row, e.x, stride, N, planar)]
                        : NV > 2 ? row_byte4(v0, v1, v2, v3, e.x) : NV > 0 ? row_byte(v0, v1, e.x)
                                 : bins[bin_off(row, e.x, stride, N, planar)];
          bool gl;
          if (b == NA_BIN) gl = (e.y >> 16) & 1;
          else if ((e.y >> 17) & 1) gl = (lv[d].dec[i].bits[b >> 5] >> (b & 31)) & 1u;
          else gl = b < (e.y & 0xFFFF);
          c = gl ? e.z : e.w;
        }
      } else {
        const Dec* dc = lv[d].dec + i;
        const int f = dc->feat;
        if (f < 0) {
          c = lv[d].cl[i];
        } else {
          c = dec_go_left_key<GRP>(dc, split_key<NV, GRP>(dc->is_cat == GROUP_CAT, f, v0, v1, v2, v3, bins, row, stride,
                                                          N, planar)) ? lv[d].cl[i] : lv[d].cr[i];
        }
      }
      if (c < 0) { leaf = -1 - c; break; }
      i = c;
    }
    leaf_of_row[row] = leaf;
    const long long qn = (long long)(a_n * sn), qd = (long long)(a_d * sd);
    if (lds) {
      if (qn) atomicAdd(sq + 2 * leaf, (unsigned long long)qn);
      if (qd) atomicAdd(sq + 2 * leaf + 1, (unsigned long long)qd);
    } else {
      unsigned long long* lq = leafq + (size_t)(blockIdx.x % LEAFQ_STRIPES) * 2 * leaf_cap;
      if (qn) atomicAdd(lq + 2 * leaf, (unsigned long long)qn);
      if (qd) atomicAdd(lq + 2 * leaf + 1, (unsigned long long)qd);
    }
  }
  if (lds) {
    __syncthreads();
    // one of LEAFQ_STRIPES copies per block (k_leafsum_finish adds them): 2048 blocks flushing into one
    // set of leaf slots serialised on those few L2 addresses (57 us of a 1.375M-row tree)
    unsigned long long* lq = leafq + (size_t)(blockIdx.x % LEAFQ_STRIPES) * 2 * leaf_cap;
    for (int i = threadIdx.x; i < 2 * leaf_cap; i += blockDim.x)
      if (sq[i]) atomicAdd(lq + i, sq[i]);
  }
}

// fixed-point leaf sums -> fp64 leafsum[L][2] (and, with leafval, the closed-form Newton leaf values of
// k_leaf_values); also re-zeroes the fixed-point slots for the next tree
struct LeafVals {       // closed-form leaf values folded into k_leafsum_finish (out == null: none)
  int log_link;
  double scale, kclamp, mx, lam, l1;
  float* out;
};

__device__ __forceinline__ float leaf_value(double num, double den, const LeafVals& v) {
  if (v.l1 > 0.0) num = num > v.l1 ? num - v.l1 : (num < -v.l1 ? num + v.l1 : 0.0);
  double g = den == 0.0 ? 0.0 : num / (den + v.lam);
  if (v.log_link) g = den == 0.0 ? 0.0 : log(fmax(g, 1e-300));
  double x = v.scale * g;
  if (x != x) x = 0.0;                                      // nan_to_num(nan=0)
  if (v.kclamp > 0.0) x = fmin(fmax(x, -v.kclamp), v.kclamp);  // multinomial +-1e4
  if (isinf(x)) x = x > 0 ? 1e4 : -1e4;                      // nan_to_num(posinf/neginf=+-1e4)
  x = fmin(fmax(x, -v.mx), v.mx);                           // max_abs_leafnode_pred (inf: no-op)
  return (float)x;
}

__device__ __forceinline__ void leafsum_one(unsigned long long* __restrict__ leafq, const double* __restrict__ qs,
                                            int n, double* __restrict__ leafsum, const LeafVals& lv, int i) {
  long long a = 0, b = 0;
  for (int k = 0; k < LEAFQ_STRIPES; ++k) {                 // n == leaf_cap: stripe k at k * 2 * n
    unsigned long long* q = leafq + (size_t)k * 2 * n;
    a += (long long)q[2 * i];
    b += (long long)q[2 * i + 1];
    q[2 * i] = 0ull;
    q[2 * i + 1] = 0ull;
  }
  leafsum[2 * i] = (double)a * qs[8];
  leafsum[2 * i + 1] = (double)b * qs[9];
  if (lv.out) lv.out[i] = leaf_value(leafsum[2 * i], leafsum[2 * i + 1], lv);   // single process: no second launch
}

__global__ void k_leafsum_finish(unsigned long long* __restrict__ leafq, const double* __restrict__ qs, int n,
                                 double* __restrict__ leafsum, LeafVals lv) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) leafsum_one(leafq, qs, n, leafsum, lv, i);
}

// k_leaf_assign with k_leafsum_finish folded into its LAST block: every block's leaf-sum atomics are ordered before
// its agent-scope RELEASE ticket on `done`; the block drawing the final ticket acquires and finishes all leaf_cap
// leaves (fp64 sums, re-zeroed fixed-point slots, closed-form values). One launch per tree instead of two.
// (FUSE is a template switch: the tail costs the unfused kernel 14 VGPRs — 34 -> 48 — and MEASURED r5 115 -> 140 us)
template <int NV, bool FUSE, bool GRP>
__global__ __launch_bounds__(256) void k_leaf_assign(
    const uint8_t* __restrict__ bins, int stride, long long N, const LevelPtrs* __restrict__ lv, int D,
    const float* __restrict__ an, const float* __restrict__ ad, const double* __restrict__ qs,
    int* __restrict__ leaf_of_row, unsigned long long* __restrict__ leafq, int leaf_cap, int n_nodes, int planar,
    const uint8_t* __restrict__ lvl2, double* __restrict__ leafsum, LeafVals vals, int* __restrict__ done) {
  leaf_assign_body<NV, GRP>(bins, stride, N, lv, D, an, ad, qs, leaf_of_row, leafq, leaf_cap, n_nodes, planar, lvl2);
  if (!FUSE || !done) return;
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  for (int i = threadIdx.x; i < leaf_cap; i += blockDim.x) leafsum_one(leafq, qs, leaf_cap, leafsum, vals, i);
  if (threadIdx.x == 0) __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------------
// k_bin_assign: X (column-major fp32 [F][N]) -> uint8 bins, row-major [N][stride] or planar [stride/32][N][32].
// Numeric: bin = #edges <= x (edges sorted, per feature `nedges` of them at edges + f*max_edges);
// categorical (iscat): bin = code (<= nedges) else NA. NaN -> NA_BIN.
// blockIdx.y = a group of 32 features whose edge tables are staged in LDS (binary searches stay on chip);
// a thread bins one row's 32 features into 8 packed dwords and writes them with 16-byte / dword stores
// (one byte store per feature was the bottleneck: 5e9 bins of a 100M x 50 frame took 99 ms).
__global__ __launch_bounds__(256) void k_bin_assign(const float* __restrict__ X, long long N, int F, int stride,
                                                    const float* __restrict__ edges, int max_edges,
                                                    const int* __restrict__ nedges, const int* __restrict__ iscat,
                                                    uint8_t* __restrict__ bins, int planar,
                                                    const int* __restrict__ xmap /*engine col -> X row, null = id*/) {
  extern __shared__ float se[];                       // [32][max_edges]
  __shared__ int sn[32], sc[32];
  const int f0 = blockIdx.y * 32;
  const int nf = min(32, stride - f0);                // multiple of 4 (stride is)
  const int nr = max(0, min(32, F - f0));             // real features in the group
  for (int i = threadIdx.x; i < nr * max_edges; i += blockDim.x)
    se[i] = edges[(size_t)f0 * max_edges + i];
  if (threadIdx.x < 32) {
    sn[threadIdx.x] = threadIdx.x < nr ? nedges[f0 + threadIdx.x] : 0;
    sc[threadIdx.x] = threadIdx.x < nr ? iscat[f0 + threadIdx.x] : 0;
  }
  __syncthreads();
  for (long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x; row < N;
       row += (long long)gridDim.x * blockDim.x) {
    uint32_t wd[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) wd[k] = 0u;
#pragma unroll
    for (int fl = 0; fl < 32; ++fl) {
      if (fl < nr) {
        const int xr = xmap ? xmap[f0 + fl] : f0 + fl;
        const float x = X[(long long)xr * N + row];
        int b;
        if (x != x) b = NA_BIN;
        else if (sc[fl]) {
          const int code = (int)x;
          b = (code >= 0 && code <= sn[fl]) ? code : NA_BIN;
        } else {
          const float* e = se + fl * max_edges;
          int lo = 0, hi = sn[fl];
          while (lo < hi) { const int mid = (lo + hi) >> 1; if (e[mid] <= x) lo = mid + 1; else hi = mid; }
          b = lo;
        }
        wd[fl >> 2] |= (uint32_t)(b & 0xFF) << (8 * (fl & 3));
      }
    }
    if (planar) {
      uint4* dst = reinterpret_cast<uint4*>(bins + ((long long)blockIdx.y * N + row) * 32);
      dst[0] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
      dst[1] = make_uint4(wd[4], wd[5], wd[6], wd[7]);
    } else {
      uint32_t* dst = reinterpret_cast<uint32_t*>(bins + row * stride + f0);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (4 * k < nf) dst[k] = wd[k];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// k_predict: score raw features through a compressed forest.
//   X: column-major fp32 [F][N]. Forest nodes (SoA): feat (-1 leaf), thr, left, right (absolute node
//   index), na_left, cat_off (-1 numeric; else word offset into cat_bits), value. tree_root[t], tree_cls[t].
//   out[N][K] += value of each tree's leaf (class tree_cls[t]).
__global__ void k_predict(const float* __restrict__ X, long long N, int K,
                          const int* __restrict__ feat, const float* __restrict__ thr,
                          const int* __restrict__ left, const int* __restrict__ right,
                          const int* __restrict__ na_left, const int* __restrict__ cat_off,
                          const unsigned* __restrict__ cat_bits, const int* __restrict__ cat_nbits,
                          const float* __restrict__ value, const int* __restrict__ tree_root,
                          const int* __restrict__ tree_cls, int n_trees, float* __restrict__ out,
                          int* __restrict__ leaf_out /*nullable [N][n_trees]*/) {
  const long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= N) return;
  for (int t = 0; t < n_trees; ++t) {
    int n = tree_root[t];
    while (feat[n] >= 0) {
      const float x = X[(long long)feat[n] * N + row];
      bool go_left;
      if (x != x) go_left = na_left[n] != 0;
      else if (cat_off[n] >= 0) {
        const int code = (int)x;
        if (code < 0 || code >= cat_nbits[n]) go_left = na_left[n] != 0;
        else go_left = (cat_bits[cat_off[n] + (code >> 5)] >> (code & 31)) & 1u;
      } else go_left = x < thr[n];
      n = go_left ? left[n] : right[n];
    }
    out[row * K + tree_cls[t]] += value[n];
    if (leaf_out) leaf_out[row * n_trees + t] = n;
  }
}

// ------------------------------------------------------------------------------------------------
// Fixed-point scales: max |w|, |wY| (int64 LDS histograms) and max |num|, |den| (int64 leaf sums) of the SoA
// aux planes aux[c * N + i] -> AMAX_SHARDS x 4 shard maxima (uint bits of non-negative floats)
__global__ __launch_bounds__(256) void k_amax(const float* __restrict__ aux, long long N, unsigned* __restrict__ amax_bits) {
  float m[4] = {0.f, 0.f, 0.f, 0.f};
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (long long)gridDim.x * blockDim.x) {
#pragma unroll
    for (int c = 0; c < 4; ++c) m[c] = fmaxf(m[c], fabsf(aux[(size_t)c * N + i]));
  }
#pragma unroll
  for (int c = 0; c < 4; ++c)
    for (int off = 32; off > 0; off >>= 1) m[c] = fmaxf(m[c], __shfl_xor(m[c], off, 64));
  __shared__ float sm[4][4];
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) for (int c = 0; c < 4; ++c) sm[c][wv] = m[c];
  __syncthreads();
  if (threadIdx.x < 4) {
    const int c = threadIdx.x;
    float v = sm[c][0];
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) v = fmaxf(v, sm[c][k]);
    atomicMax(amax_bits + 4 * (blockIdx.x & (AMAX_SHARDS - 1)) + c, __float_as_uint(v));
  }
}

// folds the AMAX_SHARDS per-shard maxima, then derives the fixed-point scales
//   qs = [sa, sb, 1/sa, 1/sb, sp, 1/sp, sn, sd, 1/sn, 1/sd]
// sa, sb: 2^40 / max (per-block int64 LDS histograms); sp: 2^30 / max|wY| (packed count|wY);
// sn, sd: 2^lb / max with 2^lb * N < 2^62 (whole-tree int64 leaf sums cannot overflow).
// Also the tree's start-of-build reset: leaf counters and the amax shards themselves once read (the next
// tree's fused step re-fills them).
__global__ __launch_bounds__(256) void k_qscale(unsigned* __restrict__ amax_bits, double* __restrict__ qs,
                                                int* __restrict__ counters, long long N, int fpack) {
  __shared__ unsigned sm[4];
  if (threadIdx.x < 4) {
    unsigned mbits = 0u;
    for (int k = 0; k < AMAX_SHARDS; ++k) mbits = max(mbits, amax_bits[4 * k + threadIdx.x]);
    sm[threadIdx.x] = mbits;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int c = threadIdx.x;
    const double m = (double)__uint_as_float(sm[c]);
    const bool ok = m > 0.0 && m == m && m < 1e300;
    if (c < 2) {
      const double sc = ok ? 1099511627776.0 / m : 1.0;   // 2^40 / max
      qs[c] = sc;
      qs[2 + c] = 1.0 / sc;
      if (c == 1) {                                        // packed wY: 2^30 / max (FPACK: 32-bit field)
        const double sp = !ok ? 1.0 : fpack ? 0.99 * 2147483648.0 / ((double)PACK_MAX * m) : 1073741824.0 / m;
        qs[4] = sp;
        qs[5] = 1.0 / sp;
      } else {                                             // packed weight field: scale, 1 / scale, shift
        const double sw = (fpack && ok) ? 0.99 * 4294967296.0 / ((double)PACK_MAX * m) : 1.0;
        qs[10] = sw;
        qs[11] = 1.0 / sw;
        qs[12] = fpack ? 32.0 : (double)PACK_SHIFT;
      }
    } else {
      int lb = 61;
      for (long long n = N; n > 0; n >>= 1) --lb;          // 2^lb * N < 2^62
      if (lb < 8) lb = 8;
      const double sc = ok ? ldexp(1.0, lb) / m : 1.0;
      qs[6 + (c - 2)] = sc;
      qs[8 + (c - 2)] = 1.0 / sc;
    }
  }
  for (int i = threadIdx.x; i < 4 * AMAX_SHARDS; i += blockDim.x) amax_bits[i] = 0u;
  if (counters && threadIdx.x < 4) counters[threadIdx.x] = 0;
}

// Leaf values of the GBM distributions with a closed-form Newton step (GBM.java fitBestConstants):
// g = num/den (0 where den == 0), log-link families take log(g); scaled by the learning rate, then
// the multinomial / max_abs_leafnode_pred clamps and nan/inf sanitising of the PyTorch path.
// lam / l1 (XGBoost Newton leaves, CalcWeight: -ThresholdL1(G, alpha) / (H + lambda), 0 where H = 0)
__global__ void k_leaf_values(const double* __restrict__ leafsum, int n, int log_link, double scale, double kclamp,
                              double mx, double lam, double l1, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const LeafVals v{log_link, scale, kclamp, mx, lam, l1, out};
  out[i] = leaf_value(leafsum[2 * i], leafsum[2 * i + 1], v);
}

// ------------------------------------------------------------------------------------------------
// k_hist_root16: the ROOT histogram of the wide-bin (AUTO = UniformAdaptive, nbins_top_level 1024) layout from a
// 16-bit fine-bin plane instead of the engine's byte columns. A wide numeric feature's n engine columns hold the
// interleaved edge subsets e[k::n] (ops/binning.py), so the sum of its n column bytes is its fine bin
// t = #{edges <= x} (NA: 1023) and column k's bin is (t - k + n - 1) / n: the root needs ONE fine histogram per
// feature, read from 2 bytes per row and feature, instead of n byte histograms from n bytes (the tiered byte layout
// spreads a feature's columns over up to 4 32-byte planes: 4 x 352 MB and 4 atomics per row and feature at 11M x 28).
// Packed modes only (one int64 plane): entry (t, slot) at (t * 16 + slot) * 8 bytes, 1024 x 16 x 8 = 128 KiB, one
// 16-wave block per CU. Block (x, y) = the tile range of the standard root pass's block x (same partial slot, so
// k_hist_reduce is unchanged) and fine plane y (16 features = 8 words per row). A word carries 2 features; rows of
// odd parity add its high half first, so the 16 lanes of a ds_add_u64 group (2 rows x 8 words) hit 16 distinct
// slots = 16 distinct bank pairs (bank = 32 (t & 1) + 2 slot). The flush rebuilds every engine column of the plane's
// features from the fine histogram (n entries per (column, bin)) into the standard [bin][F][2] partial slot.
#define R16_NB 1024
#define R16_NA 1023
#define R16_FS 16                     // fine features per plane / block
#define R16_LDS (R16_NB * R16_FS * 8 + R16_FS * 4 + 64 * 8)
template <bool UNIT>
__global__ __launch_bounds__(BLK) void k_hist_root16(
    const unsigned* __restrict__ fine32 /*[planes][N][8] words (2 x uint16)*/, const float* __restrict__ aw,
    const float* __restrict__ ay, long long N, const int* __restrict__ meta, const int* __restrict__ fcol /*[slots][4]*/,
    const int* __restrict__ fnc /*[slots]: engine columns of the slot's feature (0: empty)*/, int F,
    double* __restrict__ partials, int slot_doubles, const double* __restrict__ qs, int f32) {
  extern __shared__ __attribute__((aligned(16))) long long smem64[];
  long long* h = smem64;
  float* nayy = (float*)(smem64 + R16_NB * R16_FS);
  double* red = (double*)(nayy + R16_FS);
  const int n_tiles = meta[2];
  if (n_tiles <= 0) return;
  const int per = (n_tiles + gridDim.x - 1) / gridDim.x;
  const int t0 = blockIdx.x * per, t1 = min(n_tiles, t0 + per);
  if (t0 >= t1) return;
  const long long rb = (long long)t0 * TILE, re = min(N, (long long)t1 * TILE);
  const int ft = blockIdx.y;
  const unsigned* w32 = fine32 + (size_t)ft * (size_t)N * 8;
  const int g = threadIdx.x / LPR, j = threadIdx.x % LPR;
  const bool lead = j == 0 && ft == 0;
  const float sa = (float)qs[10], sb = (float)qs[12], sp = (float)qs[4];
  const int pshift = (int)qs[12];
  const double inv_w = qs[11], inv_p = qs[5];
  constexpr int UNR = 8;
  char* Hb = (char*)h;
  const unsigned slo = (unsigned)(2 * j) * 8u, shi = (unsigned)(2 * j + 1) * 8u;
  double wyy_blk = 0.0;
  bool acc = false;
  for (long long ws = rb; ws < re; ws += PACK_MAX) {
    const long long we = min(re, ws + PACK_MAX);
    for (int i = threadIdx.x; i < R16_NB * R16_FS; i += BLK) h[i] = 0ll;
    if (threadIdx.x < R16_FS) nayy[threadIdx.x] = 0.f;
    __syncthreads();
    float wyy = 0.f;
    for (long long base = ws; base < we; base += (long long)RPI * UNR) {
      unsigned wd[UNR];
      float yv[UNR], wv[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const long long row = min(base + g + (long long)u * RPI, we - 1);
        wd[u] = w32[(size_t)row * 8 + j];
        yv[u] = ay[row];
        wv[u] = UNIT ? 1.f : (aw ? aw[row] : 1.f);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const long long row = base + g + (long long)u * RPI;
        if (row >= we) continue;
        const long long qa = UNIT ? (1ll << PACK_SHIFT) + (long long)(int)(yv[u] * sp) : qpack(wv[u], yv[u], sp, sa, sb);
        const unsigned w = wd[u];
        const unsigned tl = w & 0xFFFFu, th = w >> 16;
        // row parity: even rows add the low feature first, odd rows the high one (distinct slots per lane group)
        const bool odd = (row & 1) != 0;
        const unsigned t_a = odd ? th : tl, t_b = odd ? tl : th;
        const unsigned s_a = odd ? shi : slo, s_b = odd ? slo : shi;
        atomicAdd((unsigned long long*)(Hb + ((t_a << 7) + s_a)), (unsigned long long)qa);
        atomicAdd((unsigned long long*)(Hb + ((t_b << 7) + s_b)), (unsigned long long)qa);
        const float yy = UNIT ? yv[u] * yv[u] : row_yy(wv[u], yv[u]);
        if (lead) wyy += yy;
        if (tl == R16_NA) atomicAdd(nayy + 2 * j, yy);
        if (th == R16_NA) atomicAdd(nayy + 2 * j + 1, yy);
      }
    }
    double v[4] = {(double)wyy, 0.0, 0.0, 0.0};
    block_sum4(v, red);
    __syncthreads();
    wyy_blk = v[0];
    // flush: every engine column of the plane's features, [bin][F][2] (count * inv_w, wY * inv_p)
    double* part = partials + (size_t)blockIdx.x * slot_doubles;
    // (a wave covers the 64 (feature, subset) columns of one bin: its stores stay inside one [F][2] bin row)
    for (int i = threadIdx.x; i < R16_FS * 4 * NBIN; i += BLK) {
      const int bin = i >> 6, sl = (i >> 2) & 15, k = i & 3;
      const int slot = ft * R16_FS + sl;
      const int n = fnc[slot];
      if (k >= n) continue;
      const int col = fcol[slot * 4 + k];
      long long q = 0;
      if (bin == NA_BIN) {
        q = h[R16_NA * R16_FS + sl];
      } else {
        // t with (t - k + n - 1) / n == bin: t = n * bin + k - m, m = 0 .. n-1, t >= 0
        for (int m = 0; m < n; ++m) {
          const int t = n * bin + k - m;
          if (t >= 0 && t < R16_NA) q += h[t * R16_FS + sl];
        }
      }
      long long c, val;
      unpack(q, c, val, pshift);
      const double dc = (double)c * inv_w, dv = (double)val * inv_p;
      const size_t e2 = (size_t)bin * 2 * F + 2 * col;
      if (f32) {
        float2* p2 = (float2*)((float*)part + e2);
        float2 o = make_float2((float)dc, (float)dv);
        if (acc) { const float2 a = *p2; o = make_float2((float)((double)a.x + dc), (float)((double)a.y + dv)); }
        *p2 = o;
      } else {
        double2* p2 = (double2*)(part + e2);
        double2 o = make_double2(dc, dv);
        if (acc) { const double2 a = *p2; o.x += a.x; o.y += a.y; }
        *p2 = o;
      }
    }
    for (int i = threadIdx.x; i < R16_FS * 4; i += BLK) {
      const int sl = i >> 2, k = i & 3, slot = ft * R16_FS + sl;
      if (k >= fnc[slot]) continue;
      const size_t e2 = (size_t)F * 2 * NBIN + fcol[slot * 4 + k];
      if (f32) put_partial((float*)part + e2, (double)nayy[sl], acc);
      else put_partial(part + e2, (double)nayy[sl], acc);
    }
    if (threadIdx.x == 0 && ft == 0) {
      const size_t e2 = (size_t)F * 2 * NBIN + F;
      if (f32) put_partial((float*)part + e2, wyy_blk, acc);
      else put_partial(part + e2, wyy_blk, acc);
    }
    acc = true;
    __syncthreads();
  }
}

// Fine planes of k_hist_root16 from the engine's planar byte bins (once per training): row r's slot s = the sum of
// the bytes of its feature's engine columns, 1023 when the feature is NA (all of its columns hold NA_BIN). One
// thread per row reads the row's 32-byte piece of every plane (coalesced) and accumulates into its LDS column.
__global__ __launch_bounds__(256) void k_fine16_build(const uint8_t* __restrict__ master, int planes, long long N,
                                                      const int* __restrict__ cslot /*[planes * 32] slot or -1*/,
                                                      int nslot, unsigned short* __restrict__ fine) {
  __shared__ unsigned short acc[64][256];
  const int tid = threadIdx.x;
  const long long row = (long long)blockIdx.x * 256 + tid;
  for (int k = 0; k < nslot; ++k) acc[k][tid] = 0;
  if (row >= N) return;
  for (int pl = 0; pl < planes; ++pl) {
    const uint4* src = (const uint4*)(master + ((size_t)pl * (size_t)N + (size_t)row) * 32);
    const uint4 v0 = src[0], v1 = src[1];
    const unsigned wd[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
    for (int c = 0; c < 32; ++c) {
      const int sl = cslot[pl * 32 + c];
      if (sl < 0) continue;
      const unsigned b = (wd[c >> 2] >> (8 * (c & 3))) & 0xFFu;
      if (b == NA_BIN) acc[sl][tid] = 0x8000;
      else acc[sl][tid] = (unsigned short)(acc[sl][tid] + b);
    }
  }
  const int p16 = (nslot + 15) / 16;
  for (int q = 0; q < p16; ++q) {
    unsigned w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      unsigned lo = 0, hi = 0;
      const int s0 = q * 16 + 2 * i, s1 = s0 + 1;
      if (s0 < nslot) { lo = acc[s0][tid]; lo = (lo & 0x8000u) ? 1023u : lo; }
      if (s1 < nslot) { hi = acc[s1][tid]; hi = (hi & 0x8000u) ? 1023u : hi; }
      w[i] = lo | (hi << 16);
    }
    uint4* dst = (uint4*)(fine + ((size_t)q * (size_t)N + (size_t)row) * 16);
    dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
    dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
  }
}

// ================================================================================================
// C ABI launchers (called through ctypes with raw device pointers and the current HIP stream).
static int hist_dbg() {   // H2O_HIST_DBG: diagnostics of the histogram pass (A/B timing only; never in a real run)
  const char* e = getenv("H2O_HIST_DBG");
  return e ? atoi(e) : 0;
}

template <bool FILT, bool PACKED, bool UNIT, bool NONA, bool BUF>
static void launch_hist4(dim3 grid, size_t lds, hipStream_t s, const void* bins, int stride, const void* aw,
                         const void* ay, const void* nodes, const void* tile_prefix, const void* meta, int F,
                         void* partials, int slot_doubles, const void* qs, const void* pdec, void* nl_out, int f32,
                         long long N, int planar, int lgw, const void* nbins_f, const void* fine_f, const void* fdir) {
#define H2O_HB(FINE_)                                                                                              \
  hipLaunchKernelGGL((k_hist_build<FILT, PACKED, UNIT, NONA, BUF, FINE_>), grid, dim3(BLK), lds, s,               \
                     (const uint8_t*)bins, stride, (const float*)aw, (const float*)ay, (const Node*)nodes,         \
                     (const int*)tile_prefix, (const int*)meta, F, (double*)partials, slot_doubles, (const double*)qs, \
                     (const Dec*)pdec, (int*)nl_out, f32, N, planar, lgw, (const int*)nbins_f, (const int*)fine_f,  \
                     (const uint8_t*)fdir, hist_dbg())
  // FINE (fine-bin atomics of aligned 4-column wide groups, off by default): a separate instantiation, so the common
  // kernels carry no per-row fine / live branch
  if (fine_f) H2O_HB(true); else H2O_HB(false);
#undef H2O_HB
}

template <bool PACKED, bool UNIT>
static void launch_hist(dim3 grid, size_t lds, hipStream_t s, const void* bins, int stride, const void* aw,
                        const void* ay, const void* nodes, const void* tile_prefix, const void* meta, int F,
                        void* partials, int slot_doubles, const void* qs, const void* pdec, void* nl_out, int f32,
                        long long N, int planar, const void* nbins_f, const void* fine_f, const void* fdir) {
  // flags: bit 0 planar bins, bit 1 no NA bin anywhere (NONA kernels)
  const bool nona = (planar >> 1) & 1;
  planar &= 1;
  // BUF: the bins buffer this kernel reads (row-major, or one 32-byte plane) and the aux planes fit 32-bit offsets
  // and the row bytes are a power of two
  const int rowb = planar ? 32 : stride;
  const unsigned long long bytes = (unsigned long long)N * (unsigned long long)rowb;
  int lgw = -1;
  for (int k = 0; k < 12; ++k) if (rowb == (1 << k)) lgw = k;
  // (buffer offsets and NUM_RECORDS are unsigned 32-bit: up to 4 GiB per buffer, e.g. a 100M-row 32-byte plane)
  const char* e_buf = getenv("H2O_HIST_BUF");     // A/B and test switch: 0 = 64-bit addressing
  const bool buf = lgw >= 0 && bytes < (1ull << 32) && (unsigned long long)N * 4ull < (1ull << 32) &&
                   !(e_buf && strcmp(e_buf, "0") == 0);
#define H2O_HIST_CASE(F_, N_, B_) \
  launch_hist4<F_, PACKED, UNIT, N_, B_>(grid, lds, s, bins, stride, aw, ay, nodes, tile_prefix, meta, F, partials, \
                                          slot_doubles, qs, pdec, nl_out, f32, N, planar, lgw, nbins_f, fine_f, fdir)
  const bool filt = pdec != nullptr;
  if (filt) {
    if (nona) { if (buf) H2O_HIST_CASE(true, true, true); else H2O_HIST_CASE(true, true, false); }
    else { if (buf) H2O_HIST_CASE(true, false, true); else H2O_HIST_CASE(true, false, false); }
  } else {
    if (nona) { if (buf) H2O_HIST_CASE(false, true, true); else H2O_HIST_CASE(false, true, false); }
    else { if (buf) H2O_HIST_CASE(false, false, true); else H2O_HIST_CASE(false, false, false); }
  }
#undef H2O_HIST_CASE
}

template <typename P, typename TO>
static void reduce_launch(const void* partials, int slot_doubles, int used, const void* nodes, const void* bp,
                          const void* meta, int cap, int grid, void* out, int ostride, void* hist_next,
                          const void* hist_cur, int lo_F, hipStream_t s) {
  const int F = (used - 1) / (2 * NBIN + 1);
  if (lo_F >= F) lo_F = 0;
  const int n = lo_F > 0 ? NBIN * 2 * lo_F + F + 1 : used;
  // many node slots at this level (>= 16: a built node's rows span <= ~1/8 of the grid): column-wave form
  if (cap >= 16 && !getenv("H2O_REDUCE_SPLIT")) {
    const int gx = (n + 64 * RW - 1) / (64 * RW);
    hipLaunchKernelGGL((k_hist_reduce<P, TO, true>), dim3(gx, cap), dim3(RW * 64), 0, s, (const P*)partials,
                       slot_doubles, used, (const Node*)nodes, (const int*)bp, (const int*)meta, grid, (TO*)out,
                       ostride, (double*)hist_next, (const double*)hist_cur, lo_F);
    return;
  }
  const int gx = (n + 63) / 64;
  hipLaunchKernelGGL((k_hist_reduce<P, TO, false>), dim3(gx, cap), dim3(RW * 64), 0, s, (const P*)partials, slot_doubles,
                     used, (const Node*)nodes, (const int*)bp, (const int*)meta, grid, (TO*)out, ostride,
                     (double*)hist_next, (const double*)hist_cur, lo_F);
}

extern "C" {

int h2o_abi_version() { return H2O_ABI_VERSION; }

int h2o_tree_sizes(int* out) {
  out[7] = AMAX_SHARDS;
  out[8] = LEAFQ_STRIPES;
  out[0] = sizeof(Node); out[1] = sizeof(Dec); out[2] = sizeof(Cand); out[3] = TILE; out[4] = FTILE;
  out[5] = HIST_LDS_BYTES + HIST_LDS_TAIL;  // k_hist_build LDS bytes
  out[6] = BLK;
  return 0;
}

// partials: >= (grid + max nodes of the level) slots of slot_doubles. nbins_f (nullable): per-feature bin counts,
// which let NONA launches spread the updates of low-cardinality features over copies of their bins. fine_f
// (nullable): 1 for the columns of word-aligned 4-column wide numeric groups (one fine atomic per row and group).
// nft_lim > 0: only the first nft_lim feature tiles (planes) are built (narrow levels; the slot layout stays F)
int h2o_hist_build(const void* bins, int stride, const void* aw, const void* ay, const void* nodes,
                   const void* tile_prefix, const void* meta, int F, void* partials, int slot_doubles, const void* qs,
                   int grid, int packed, const void* pdec, void* nl_out, int f32, long long N, int planar,
                   const void* nbins_f, const void* fine_f, int nft_lim, const void* fdir, hipStream_t s) {
  int nft = (F + FTILE - 1) / FTILE;
  if (nft_lim > 0 && nft_lim < nft) nft = nft_lim;
  // A/B switches: H2O_HIST_REPL=0 drops the low-cardinality bin replicas, H2O_HIST_FINE=1 enables the
  // fine-bin atomics of 4-column wide groups (MEASURED slower: AUTO 11M plain pass 482 vs 325 us, r4)
  const char* e_repl = getenv("H2O_HIST_REPL");
  const char* e_fine = getenv("H2O_HIST_FINE");
  const bool repl = !e_repl || strcmp(e_repl, "0") != 0;
  const bool fine = e_fine && strcmp(e_fine, "1") == 0;
  if (!repl) nbins_f = nullptr;
  if (!fine) fine_f = nullptr;
  // packed mode needs one int64 plane (66 KB): two 16-wave blocks share a CU (32 waves, 8 per SIMD)
  const size_t lds = (packed ? HIST_LDS_BYTES - HPLANE * 8 : HIST_LDS_BYTES) + HIST_LDS_TAIL;
  const dim3 gr(grid, nft);
  if (packed && aw == nullptr)   // unit row weights (the trainer dropped the w plane)
    launch_hist<true, true>(gr, lds, s, bins, stride, aw, ay, nodes, tile_prefix, meta, F, partials, slot_doubles, qs, pdec, nl_out, f32, N, planar, nbins_f, fine_f, fdir);
  else if (packed) launch_hist<true, false>(gr, lds, s, bins, stride, aw, ay, nodes, tile_prefix, meta, F, partials, slot_doubles, qs, pdec, nl_out, f32, N, planar, nbins_f, fine_f, fdir);
  else launch_hist<false, false>(gr, lds, s, bins, stride, aw, ay, nodes, tile_prefix, meta, F, partials, slot_doubles, qs, pdec, nl_out, f32, N, planar, nbins_f, fine_f, fdir);
  return (int)hipGetLastError();
}


// fine: [ceil(nslot / 16)][N][16] uint16 (see k_fine16_build); nslot <= 64
int h2o_fine16_build(const void* master, int planes, long long N, const void* cslot, int nslot, void* fine,
                     hipStream_t s) {
  if (nslot < 1 || nslot > 64 || planes < 1 || N <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_fine16_build, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, (const uint8_t*)master, planes,
                     N, (const int*)cslot, nslot, (unsigned short*)fine);
  return (int)hipGetLastError();
}

// Root histogram from the 16-bit fine planes (k_hist_root16): packed modes only (packed 1 / 2); planes = slots / 16.
int h2o_hist_root16(const void* fine, int planes, const void* aw, const void* ay, long long N, const void* meta,
                    const void* fcol, const void* fnc, int F, void* partials, int slot_doubles, const void* qs, int grid,
                    int f32, hipStream_t s) {
  if (planes < 1 || grid < 1 || N <= 0) return (int)hipErrorInvalidValue;
  const dim3 gr(grid, planes);
  if (aw == nullptr)
    hipLaunchKernelGGL((k_hist_root16<true>), gr, dim3(BLK), R16_LDS, s, (const unsigned*)fine, (const float*)aw,
                       (const float*)ay, N, (const int*)meta, (const int*)fcol, (const int*)fnc, F, (double*)partials,
                       slot_doubles, (const double*)qs, f32);
  else
    hipLaunchKernelGGL((k_hist_root16<false>), gr, dim3(BLK), R16_LDS, s, (const unsigned*)fine, (const float*)aw,
                       (const float*)ay, N, (const int*)meta, (const int*)fcol, (const int*)fnc, F, (double*)partials,
                       slot_doubles, (const double*)qs, f32);
  return (int)hipGetLastError();
}

// grid: the G the matching h2o_hist_build ran with; out / hist_next may be null (see k_hist_reduce).
// out: compact build slots of ostride values (0: slot_doubles), fp32 when out_f32 (the exchange's wire dtype)
// lo_F > 0 (narrow level): only the entries of columns < lo_F (and the NA / node tails) are summed
int h2o_hist_reduce(const void* partials, int slot_doubles, int used, const void* nodes, const void* bp,
                    const void* meta, int cap, int grid, void* out, void* hist_next, const void* hist_cur,
                    int f32, int out_f32, int ostride, int lo_F, hipStream_t s) {
  if (ostride <= 0) ostride = slot_doubles;
  if (f32 && out_f32)
    reduce_launch<float, float>(partials, slot_doubles, used, nodes, bp, meta, cap, grid, out, ostride, hist_next, hist_cur, lo_F, s);
  else if (f32)
    reduce_launch<float, double>(partials, slot_doubles, used, nodes, bp, meta, cap, grid, out, ostride, hist_next, hist_cur, lo_F, s);
  else if (out_f32)
    reduce_launch<double, float>(partials, slot_doubles, used, nodes, bp, meta, cap, grid, out, ostride, hist_next, hist_cur, lo_F, s);
  else
    reduce_launch<double, double>(partials, slot_doubles, used, nodes, bp, meta, cap, grid, out, ostride, hist_next, hist_cur, lo_F, s);
  return (int)hipGetLastError();
}

int h2o_leaf_values(const void* leafsum, int n, int log_link, double scale, double kclamp, double mx, double lam,
                    double l1, void* out,
                    hipStream_t s) {
  hipLaunchKernelGGL(k_leaf_values, dim3((n + 255) / 256), dim3(256), 0, s, (const double*)leafsum, n, log_link,
                     scale, kclamp, mx, lam, l1, (float*)out);
  return (int)hipGetLastError();
}

static int split_find_launch(void* hist, int slot_doubles, const void* meta, int cap, int F, const void* nbins_f,
                             const void* iscat_f, const void* mono_f, const SplitParams& p, int level, void* cand,
                             void* root_w, const void* edges, int adapt_nb, int f0, int FL, Derive dv, hipStream_t s) {
  if (F <= 0 || cap <= 0) return 0;
  if (FL < F) return (int)hipErrorInvalidValue;
  if (p.gcat)
    hipLaunchKernelGGL(k_split_find<true>, dim3(cap, F), dim3(256), 0, s, (double*)hist, slot_doubles,
                       (const int*)meta, F, (const int*)nbins_f, (const int*)iscat_f, (const int*)mono_f, p, level,
                       (Cand*)cand, (double*)root_w, (const float*)edges, adapt_nb, f0, FL, dv);
  else
    hipLaunchKernelGGL(k_split_find<false>, dim3(cap, F), dim3(256), 0, s, (double*)hist, slot_doubles,
                       (const int*)meta, F, (const int*)nbins_f, (const int*)iscat_f, (const int*)mono_f, p, level,
                       (Cand*)cand, (double*)root_w, (const float*)edges, adapt_nb, f0, FL, dv);
  return (int)hipGetLastError();
}

int h2o_split_find(const void* hist, int slot_doubles, const void* meta, int cap, int F, const void* nbins_f,
                   const void* iscat_f, const void* mono_f, double min_w, double msi, double lambda_, double alpha,
                   double gamma, int mode, int random_split, unsigned long long seed, int level, void* cand,
                   void* root_w, const void* edges, int adapt_nb, int hist_type, int f0, int FL, hipStream_t s) {
  SplitParams p;
  p.min_w = min_w; p.min_split_improvement = msi; p.lambda = lambda_; p.alpha = alpha; p.gamma = gamma;
  p.mode = mode; p.random_split = random_split; p.seed = seed; p.hist_type = hist_type; p.fcut = 0;
  p.vrange = nullptr; p.hprev = nullptr; p.pdec = nullptr; p.rnodes = nullptr; p.fgroup = nullptr; p.edges_all = nullptr;
  p.range_on = 0; p.pad_r = 0; p.gcat = nullptr;
  return split_find_launch((void*)hist, slot_doubles, meta, cap, F, nbins_f, iscat_f, mono_f, p, level, cand, root_w,
                           edges, adapt_nb, f0, FL, Derive{nullptr, 0, 0, nullptr, nullptr}, s);
}

int h2o_split_reduce(const void* cand, const void* meta, int cap, int F, const void* feat_ok, int k_cols,
                     unsigned long long seed, int level, void* dec, const void* node_ok, const void* fgroup,
                     int cfs, hipStream_t s) {
  hipLaunchKernelGGL(k_split_reduce, dim3(cap), dim3(64), 0, s, (const Cand*)cand, (const int*)meta, F,
                     (const int*)feat_ok, k_cols, seed, level, (Dec*)dec, (const unsigned char*)node_ok,
                     (const int*)fgroup, cfs, cap);
  return (int)hipGetLastError();
}

int h2o_ic_next(const void* next, const void* next_meta, const void* dec, const void* ok_cur, const void* ic_map, int F,
                void* ok_next, int cap_next, hipStream_t s) {
  if (cap_next <= 0) return 0;
  hipLaunchKernelGGL(k_ic_next, dim3(cap_next), dim3(64), 0, s, (const Node*)next, (const int*)next_meta,
                     (const Dec*)dec, (const unsigned char*)ok_cur, (const unsigned char*)ic_map, F,
                     (unsigned char*)ok_next);
  return (int)hipGetLastError();
}

static int plan_wave_off() {
  static int v = -1;
  if (v < 0) { const char* e = getenv("H2O_PLAN_WAVE"); v = (e && e[0] == '0') ? 1 : 0; }
  return v;
}

static int plan_launch(const void* nodes, const void* meta, void* dec, void* node_nl, const void* prev_nl, void* curs,
                       void* child_l, void* child_r, void* next, void* next_tile_prefix, void* next_meta,
                       void* next_build_prefix, void* counters, void* scratch, int depth, int max_depth, double min_w,
                       int cap_next, int leaf_cap, PlanReduce pr, hipStream_t s) {
  pr.no_wave = plan_wave_off();
  hipLaunchKernelGGL(k_plan, dim3(1), dim3(1024), 0, s, (const Node*)nodes, (const int*)meta, (Dec*)dec,
                     (int*)node_nl, (const int*)prev_nl, (int4*)curs, (int*)child_l, (int*)child_r, (Node*)next,
                     (int*)next_tile_prefix, (int*)next_meta, (int*)next_build_prefix, (int*)counters, (int*)scratch,
                     depth, max_depth, min_w, cap_next, leaf_cap, pr);
  return (int)hipGetLastError();
}

int h2o_plan(const void* nodes, const void* meta, const void* dec, void* node_nl, const void* prev_nl, void* curs,
             void* child_l, void* child_r, void* next, void* next_tile_prefix, void* next_meta, void* next_build_prefix,
             void* counters, void* scratch, int depth, int max_depth, double min_w, int cap_next, int leaf_cap,
             hipStream_t s) {
  PlanReduce pr{nullptr, 0, nullptr, 0, 0ull, nullptr, nullptr, 0, 0};
  return plan_launch(nodes, meta, (void*)dec, node_nl, prev_nl, curs, child_l, child_r, next, next_tile_prefix,
                     next_meta, next_build_prefix, counters, scratch, depth, max_depth, min_w, cap_next, leaf_cap, pr, s);
}

int h2o_ranges(void* next, const void* curs, void* tp, void* bp, void* meta, hipStream_t s) {
  hipLaunchKernelGGL(k_ranges, dim3(1), dim3(1024), 0, s, (Node*)next, (const int4*)curs, (int*)tp, (int*)bp,
                     (int*)meta);
  return (int)hipGetLastError();
}

int h2o_zero_hist(void* hist, const void* next, const void* meta, int cap, int slot_doubles, hipStream_t s) {
  const int gx = (slot_doubles + 1023) / 1024;
  hipLaunchKernelGGL(k_zero_hist, dim3(gx < 64 ? gx : 64, cap), dim3(256), 0, s, (double*)hist,
                     (const Node*)next, (const int*)meta, slot_doubles);
  return (int)hipGetLastError();
}


// out_f32: write the packed slices as fp32 (the wire format of the sliced exchange)
int h2o_hist_pack(const void* src, int slot, int F, int Fs, int W, int n, void* dst, int out_f32, hipStream_t s) {
  if (n <= 0) return 0;
  const long long total = (long long)W * n * ((long long)Fs * 2 * NBIN + Fs + 1);
  long long g = (total + 255) / 256;
  const dim3 gr((unsigned)(g < 4096 ? g : 4096));
  if (out_f32)
    hipLaunchKernelGGL(k_hist_pack<float>, gr, dim3(256), 0, s, (const double*)src, slot, F, Fs, W, n, (float*)dst);
  else
    hipLaunchKernelGGL(k_hist_pack<double>, gr, dim3(256), 0, s, (const double*)src, slot, F, Fs, W, n, (double*)dst);
  return (int)hipGetLastError();
}

static bool route_generic() {   // H2O_ROUTE_GENERIC=1: byte-load path (A/B measurements)
  static int v = -1;
  if (v < 0) { const char* e = getenv("H2O_ROUTE_GENERIC"); v = (e && e[0] == '1') ? 1 : 0; }
  return v == 1;
}

static int nv_of(int stride) {
  if (route_generic()) return 0;
  return stride == 64 ? 4 : stride == 48 ? 3 : stride == 32 ? 2 : stride == 16 ? 1 : 0;
}

// regroup an even level two levels down (moving bins + wY (+ w) of continuing rows)
// lp > 0 (planar): only the first lp (1 or 2) planes of each row move — the narrow levels below read no other
// column; split bytes of columns past them (the decisions of the levels above) are read from the source
// lvl2 (nullable; the root route only): per ORIGINAL row its level-2 node, or 128 + its leaf (k_leaf_assign
// starts there)
static int route_launch(const void* sbins, const void* say, const void* saw, void* dbins, void* day, void* daw,
                        int stride, const void* nodesA, const void* tpA, const void* metaA, const void* decA,
                        const void* clA, const void* crA, const void* decB, const void* clB, const void* crB,
                        void* curs, int tiles_cap, long long N, int planar, int lp, void* lvl2, const void* fdir,
                        RangesOut ro, hipStream_t s, int grp = 0) {
  if (planar && (stride % 32 != 0 || stride < 64)) return (int)hipErrorInvalidValue;
  if (lp < 0 || lp > 2 || (lp > 0 && !planar)) return (int)hipErrorInvalidValue;
#define ROUTE_LAUNCH(NV) do { if (grp) ROUTE_LAUNCH2(NV, true); else ROUTE_LAUNCH2(NV, false); } while (0)
#define ROUTE_LAUNCH2(NV, G)                                                                                   \
  hipLaunchKernelGGL((k_route<NV, G>), dim3(tiles_cap), dim3(LW * 64), 0, s, (const uint8_t*)sbins,           \
                     (const float*)say, (const float*)saw, (uint8_t*)dbins, (float*)day, (float*)daw, stride,  \
                     (const Node*)nodesA, (const int*)tpA, (const int*)metaA, (const Dec*)decA, (const int*)clA, \
                     (const int*)crA, (const Dec*)decB, (const int*)clB, (const int*)crB, (int4*)curs, N, planar, \
                     (uint8_t*)lvl2, (const uint8_t*)fdir, ro)
  switch (lp == 1 ? 2 : lp == 2 ? 4 : nv_of(stride)) {
    case 4: ROUTE_LAUNCH(4); break;
    case 3: ROUTE_LAUNCH(3); break;
    case 2: ROUTE_LAUNCH(2); break;
    case 1: ROUTE_LAUNCH(1); break;
    default: ROUTE_LAUNCH(0);
  }
#undef ROUTE_LAUNCH
#undef ROUTE_LAUNCH2
  return (int)hipGetLastError();
}

int h2o_route(const void* sbins, const void* say, const void* saw, void* dbins, void* day, void* daw, int stride,
              const void* nodesA, const void* tpA, const void* metaA, const void* decA, const void* clA,
              const void* crA, const void* decB, const void* clB, const void* crB, void* curs, int tiles_cap,
              long long N, int planar, int lp, void* lvl2, const void* fdir, hipStream_t s) {
  return route_launch(sbins, say, saw, dbins, day, daw, stride, nodesA, tpA, metaA, decA, clA, crA, decB, clB, crB,
                      curs, tiles_cap, N, planar, lp, lvl2, fdir, RangesOut{nullptr, nullptr, nullptr, nullptr, nullptr},
                      s);
}

// leaf id of every row (original order) + fixed-point leaf sums -> fp64 leafsum[leaf_cap][2]
static int leaf_assign_launch(const void* master, int stride, long long N, const void* lvptrs, int D, const void* an,
                              const void* ad, const void* qs, void* leaf_of_row, void* leafq, int leaf_cap,
                              void* leafsum, int n_nodes, int planar, LeafVals lv, hipStream_t s,
                              const void* lvl2 = nullptr, int* done = nullptr, int grp = 0) {
  if (D > TP_MAXL_DEV) return (int)hipErrorInvalidValue;
  long long grid = (N + 255) / 256;
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  const size_t lds = (leaf_cap <= LEAF_LDS_MAX ? (size_t)16 * leaf_cap : 0) +
                     (n_nodes <= LEAF_TREE_MAX ? (size_t)16 * n_nodes : 0);
#define LA(NV) do { if (done) { LA1(NV, true); } else { LA1(NV, false); } } while (0)
#define LA1(NV, FU) do { if (grp) { LA2(NV, FU, true); } else { LA2(NV, FU, false); } } while (0)
#define LA2(NV, FU, G) hipLaunchKernelGGL((k_leaf_assign<NV, FU, G>), dim3((unsigned)grid), dim3(256), lds, s, (const uint8_t*)master, \
                                  stride, N, (const LevelPtrs*)lvptrs, D, (const float*)an, (const float*)ad,          \
                                  (const double*)qs, (int*)leaf_of_row, (unsigned long long*)leafq, leaf_cap, n_nodes, planar, \
                                  (const uint8_t*)lvl2, (double*)leafsum, lv, done)
  // planar rows of more than two planes: with the root route's level-2 positions (narrow levels below) only the
  // first plane in registers, else the first two; split bytes of later planes are loaded per level
  switch ((planar && stride > 64 && !route_generic()) ? (lvl2 ? 2 : 4) : nv_of(stride)) {
    case 4: LA(4); break;
    case 3: LA(3); break;
    case 2: LA(2); break;
    case 1: LA(1); break;
    default: LA(0);
  }
#undef LA
#undef LA1
#undef LA2
  if (!done)
    hipLaunchKernelGGL(k_leafsum_finish, dim3((leaf_cap + 255) / 256), dim3(256), 0, s, (unsigned long long*)leafq,
                       (const double*)qs, leaf_cap, (double*)leafsum, lv);
  return (int)hipGetLastError();
}

int h2o_leaf_assign(const void* master, int stride, long long N, const void* lvptrs, int D, const void* an,
                    const void* ad, const void* qs, void* leaf_of_row, void* leafq, int leaf_cap, void* leafsum,
                    int n_nodes, int planar, hipStream_t s) {
  const LeafVals lv{0, 0.0, 0.0, 0.0, 0.0, 0.0, nullptr};
  return leaf_assign_launch(master, stride, N, lvptrs, D, an, ad, qs, leaf_of_row, leafq, leaf_cap, leafsum, n_nodes,
                            planar, lv, s);
}

int h2o_amax(const void* aux, long long N, void* amax_bits, hipStream_t s) {
  long long grid = (N + 255) / 256;
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_amax, dim3((unsigned)grid), dim3(256), 0, s, (const float*)aux, N, (unsigned*)amax_bits);
  return (int)hipGetLastError();
}

// Tree snapshot to pinned host memory from a kernel (the arena's 16-byte words stored straight into the mapped
// host buffer) instead of a runtime device-to-host copy. (r5 A/B: the runtime copy started ~12 us after the last
// tree kernel in every tree.)
__global__ __launch_bounds__(256) void k_snap_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, long long n16,
                                                   const unsigned char* __restrict__ srcb, unsigned char* __restrict__ dstb,
                                                   long long nbytes) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (long long)gridDim.x * blockDim.x)
    dst[i] = src[i];
  const long long t = n16 * 16 + (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < nbytes) dstb[t] = srcb[t];
}

// device address of a pinned host buffer (hipHostGetDevicePointer); nonzero return: not mapped for the device
int h2o_host_dev_ptr(void* host, unsigned long long* out) {
  void* d = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&d, host, 0);
  *out = (unsigned long long)(uintptr_t)d;
  return (int)e;
}

int h2o_snap_copy(const void* src, void* dst, long long nbytes, hipStream_t s) {
  if (nbytes <= 0) return 0;
  if ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) return (int)hipErrorInvalidValue;
  const long long n16 = nbytes / 16;
  long long grid = (n16 + 255) / 256;
  if (grid < 1) grid = 1;
  if (grid > 64) grid = 64;
  hipLaunchKernelGGL(k_snap_copy, dim3((unsigned)grid), dim3(256), 0, s, (const uint4*)src, (uint4*)dst, n16,
                     (const unsigned char*)src, (unsigned char*)dst, nbytes);
  return (int)hipGetLastError();
}

int h2o_qscale(void* amax_bits, void* qs, void* counters, long long N, int fpack, hipStream_t s) {
  hipLaunchKernelGGL(k_qscale, dim3(1), dim3(256), 0, s, (unsigned*)amax_bits, (double*)qs, (int*)counters, N, fpack);
  return (int)hipGetLastError();
}

int h2o_bin_assign(const void* X, long long N, int F, int stride, const void* edges, int max_edges,
                   const void* nedges, const void* iscat, void* bins, int planar, const void* xmap,
                   hipStream_t s) {
  if (planar && (stride % 32 != 0 || stride < 64)) return (int)hipErrorInvalidValue;
  if (stride % 4 != 0 || max_edges < 1 || (size_t)32 * max_edges * sizeof(float) > 96 * 1024)
    return (int)hipErrorInvalidValue;
  const int blk = 256;
  const int groups = (stride + 31) / 32;
  long long grid = (N + blk - 1) / blk;
  if (grid > 4096) grid = 4096;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_bin_assign, dim3((unsigned)grid, (unsigned)groups), dim3(blk),
                     (size_t)32 * max_edges * sizeof(float), s, (const float*)X, N, F, stride,
                     (const float*)edges, max_edges, (const int*)nedges, (const int*)iscat, (uint8_t*)bins, planar,
                     (const int*)xmap);
  return (int)hipGetLastError();
}

int h2o_predict(const void* X, long long N, int K, const void* feat, const void* thr, const void* left,
                const void* right, const void* na_left, const void* cat_off, const void* cat_bits,
                const void* cat_nbits, const void* value, const void* tree_root, const void* tree_cls, int n_trees,
                void* out, void* leaf_out, hipStream_t s) {
  const int blk = 256;
  const long long grid = (N + blk - 1) / blk;
  hipLaunchKernelGGL(k_predict, dim3((unsigned)grid), dim3(blk), 0, s, (const float*)X, N, K, (const int*)feat,
                     (const float*)thr, (const int*)left, (const int*)right, (const int*)na_left,
                     (const int*)cat_off, (const unsigned*)cat_bits, (const int*)cat_nbits, (const float*)value,
                     (const int*)tree_root, (const int*)tree_cls, n_trees, (float*)out, (int*)leaf_out);
  return (int)hipGetLastError();
}


// ================================================================================================
// Native per-tree launch sequence: a tree costs a handful of host calls instead of ~45 ctypes round trips
// (at 1.375M rows/GPU the Python launch loop alone took ~370 us/tree and left the GPU 18 % idle).
// Row-sharded runs use h2o_tree_dist: the same launches with the level collectives enqueued in between.
// Aux planes are SoA (aux[c * N + i]: 0 = w (null-able: unit weights), 1 = wY, 2 = gamma numerator,
// 3 = gamma denominator); the routed ping-pong buffers carry bins + wY (+ w).
#define TP_MAXL 65
struct TreePlan {
  long long N;
  int stride, F, D, slot, used, pf32, grid, leaf_cap, mode, random_split, unit;
  double min_w, msi, lam, alpha, gamma;
  void *master, *partials, *hist0, *hist1, *hbuild, *cand, *scratch, *nbins_f, *iscat_f, *mono_f;
  void *qs, *leafsum, *leaf_of_row, *counters, *rootw, *leafval, *leafq, *lvptrs;
  void *bb[2], *by[2], *bw[2];
  void *nodes[TP_MAXL], *meta[TP_MAXL], *tp[TP_MAXL], *bp[TP_MAXL], *dec[TP_MAXL], *cl[TP_MAXL], *cr[TP_MAXL],
      *nl[TP_MAXL], *cur[TP_MAXL];
  int caps[TP_MAXL], tiles_cap[TP_MAXL];
  // per tree
  void *aux, *amax_bits, *feat_ok;
  int compute_amax, k_cols, packed, leaf_native, log_link, hist_type;
  unsigned long long seed;
  double scale, kclamp, mx;
  int kc_level[TP_MAXL];   // per-level column sample size (col_sample_rate_change_per_level); 0 = k_cols
  int pad2;
  void* edges;             // [F][255] global bin edges for UniformAdaptive candidates (null: QuantilesGlobal)
  int nb_level[TP_MAXL];   // UniformAdaptive bins per level (0 = off)
  int pad3;
  void* ic_map;            // [F][F] interaction-constraint map (null: no constraints)
  void* ic[TP_MAXL];       // per level [caps][F] allowed-feature masks (ic[0] = the root's)
  // feature-sliced row-sharded mode (sliced = 1): this rank searches features [fs0, fs0 + fsn) of histograms
  // whose slots hold only the slice (sslot doubles, k_hist_pack layout); candidates go to cand_local
  // [cap][fsn] and the caller all-gathers them into cand [cap][F]. hrecv = reduce-scattered build slots.
  int sliced, fs0, fsn, sslot;
  void *cand_local, *hrecv;
  double leaf_lam, leaf_l1;   // k_leaf_values regularisation (XGBoost leaves; 0 for GBM)
  int planar, no_na;          // bins layout of master and the ping-pong buffers (see bin_off); no_na: no NA bin
                              // anywhere in the bins (the histogram loop skips its per-word NA test)
  void* fgroup;               // [F] engine column -> original feature (null: identity), k_split_reduce
  // collective transport of a row-sharded tree (h2o_tree_dist): coll_fn(coll_ctx, op, send, recv, count, dtype,
  // stream), see h2o_coll_fn. RCCL (h2o_rccl_coll + an ncclComm_t) on a GPU node; a host callback under gloo.
  void* coll_fn;
  void* coll_ctx;
  int W, cf32;                // ranks; cf32: exchanged histograms travel as fp32 (half the bytes)
  int cand_fs;                // features per rank of the rank-major candidate all-gather (sliced)
  int dist;                   // row-sharded (h2o_tree_dist): build slots go out in the exchange's layout
  void *hsend, *cand_all, *lsx;  // [W][n][E] packed send slots, [W][cap][Fs] candidates, leaf sums + root weight
  void* fine_f;               // [F] int32: columns of word-aligned 4-column wide numeric groups (or null)
  // narrow levels of wide numeric bins (ops/binning.py layout: columns [0, lo_F) hold every feature's first
  // column, [lo_F, mid_F) the subsets that halve the edge spacing, the rest follow): from level lo_from on
  // (adaptive bin count <= 256) only columns < lo_F, from mid_from on (<= 512) only columns < mid_F are
  // histogrammed, reduced and searched, and the routes that feed such levels move only the planes holding them.
  // lo_F / mid_F = 0: off.
  int lo_F, lo_from, mid_F, mid_from;
  void* lvl2;                 // [N] uint8: the root route's level-2 node / 128 + leaf per row (narrow runs; or null)
  void* fdir;                 // [N] uint8: the root split's side per row (k_row_dir; narrow planar runs, or null)
  int num_plane, pad4;        // aux plane of the leaf-sum numerator (2; 1 when the step kernel elides num == wY)
  // root pass of the wide-bin layout from 16-bit fine planes (k_hist_root16; packed modes; null: the byte columns)
  void* fine16;               // [f16_planes][N][16] uint16 fine bins per original feature
  void* f16col;               // [f16_planes * 16][4] int32: engine column of subset k (or -1)
  void* f16n;                 // [f16_planes * 16] int32: the feature's engine columns (0: empty slot)
  int f16_planes, pad5;
  // the reference's node ranges of the adaptive lattices (SplitParams.range_on / vrange): [F][2] exact column extremes
  void* vrange;
  int range_on, pad6;
  void* gcat;                 // [F] wide-categorical groups (SplitParams.gcat), or null
};

// node-range fields of a level's split search (see SplitParams)
static inline void tp_node_range(const TreePlan* P, int d, const void* hprev, SplitParams& p) {
  p.range_on = (P->range_on && P->vrange && P->edges && P->nb_level[d] > 1) ? 1 : 0;
  p.vrange = (const float*)P->vrange;
  p.hprev = d > 0 ? (const double*)hprev : nullptr;
  p.pdec = d > 0 ? (const Dec*)P->dec[d - 1] : nullptr;
  p.rnodes = (const Node*)P->nodes[d];
  p.fgroup = (const int*)P->fgroup;
  p.edges_all = (const float*)P->edges;
  p.pad_r = 0;
  p.gcat = (const int*)P->gcat;
}

// op codes / dtypes of the collective transport
enum { H2O_COLL_ALLREDUCE = 0, H2O_COLL_REDUCE_SCATTER = 1, H2O_COLL_ALLGATHER = 2 };
enum { H2O_DT_F32 = 0, H2O_DT_F64 = 1, H2O_DT_U8 = 2 };
// count: ALLREDUCE elements, REDUCE_SCATTER elements received per rank, ALLGATHER elements sent per rank
typedef int (*h2o_coll_fn)(void* ctx, int op, const void* send, void* recv, long long count, int dtype,
                           hipStream_t s);

static inline const float* tp_aux(const TreePlan* P, int c) { return (const float*)P->aux + (size_t)c * P->N; }

// level e's row buffers: the master order (e == 0) or ping-pong buffer (e/2 - 1) % 2
static inline void tp_level_buf(const TreePlan* P, int e, const void*& b, const void*& y, const void*& w) {
  if (e == 0) { b = P->master; y = tp_aux(P, 1); w = P->unit ? nullptr : tp_aux(P, 0); return; }
  const int i = (e / 2 - 1) % 2;
  b = P->bb[i]; y = P->by[i]; w = P->unit ? nullptr : P->bw[i];
}

// columns level d searches (0 = all) and the planes (feature tiles) holding them
static inline int tp_fcut(const TreePlan* P, int d) {
  if (P->lo_F > 0 && d >= P->lo_from) return P->lo_F;
  if (P->mid_F > 0 && d >= P->mid_from) return P->mid_F;
  return 0;
}
static inline int tp_planes(int fc) { return fc > 0 ? (fc + FTILE - 1) / FTILE : 0; }
// the root route records every row's level-2 position when the levels below are narrow and planar (the leaf walk
// then skips the two levels whose split bytes live in other planes)
static inline void* tp_lvl2(const TreePlan* P) {
  return (P->lvl2 && P->planar && P->D > 2 && tp_fcut(P, 2) > 0 && tp_fcut(P, 2) <= FTILE) ? P->lvl2 : nullptr;
}

// fused: the route's last block also turns the final cursors into level e+2's ranges and tile prefixes (k_ranges)
static bool route_fused_ranges() {
  static int v = -1;
  if (v < 0) { const char* e = getenv("H2O_ROUTE_RANGES"); v = (e && e[0] == '0') ? 0 : 1; }
  return v == 1;
}

static int tp_route(const TreePlan* P, int e, hipStream_t s, bool ranges) {
  const void *sb, *sy, *sw;
  tp_level_buf(P, e, sb, sy, sw);
  const int di = (e / 2) % 2;
  // rows of level e + 2 (and below) are read by narrow levels only: move just the low planes
  const int np = tp_planes(tp_fcut(P, e + 2));
  const int lp = (P->planar && np <= 2) ? np : 0;
  const RangesOut ro = ranges ? RangesOut{(Node*)P->nodes[e + 2], (int*)P->tp[e + 2], (int*)P->bp[e + 2],
                                          (int*)P->meta[e + 2], (int*)P->counters + 1}
                              : RangesOut{nullptr, nullptr, nullptr, nullptr, nullptr};
  return route_launch(sb, sy, sw, P->bb[di], P->by[di], P->unit ? nullptr : P->bw[di], P->stride, P->nodes[e], P->tp[e],
                      P->meta[e], P->dec[e], P->cl[e], P->cr[e], P->dec[e + 1], P->cl[e + 1], P->cr[e + 1],
                      P->cur[e + 1], P->tiles_cap[e], P->N, P->planar, lp, e == 0 ? tp_lvl2(P) : nullptr,
                      (e == 0 && tp_lvl2(P) && P->fdir) ? P->fdir : nullptr, ro, s, P->gcat != nullptr);
}

#define TP_CHECK(x) do { int rc_ = (x); if (rc_) return rc_; } while (0)

int h2o_tree_plan_size() { return (int)sizeof(TreePlan); }

// qscale reset + root histogram (into hist0; the caller all-reduces it when row-sharded; sliced: into
// hbuild slot 0, which the caller packs and reduce-scatters into hist0)
int h2o_tree_root(const TreePlan* P, hipStream_t s) {
  if (P->D >= TP_MAXL - 1) return (int)hipErrorInvalidValue;
  if (P->compute_amax) TP_CHECK(h2o_amax(P->aux, P->N, P->amax_bits, s));
  TP_CHECK(h2o_qscale(P->amax_bits, P->qs, P->counters, P->N, P->packed == 2, s));
  const int g0 = P->tiles_cap[0] < P->grid ? P->tiles_cap[0] : P->grid;
  if (P->fine16 && P->packed && !P->sliced && tp_fcut(P, 0) == 0)
    TP_CHECK(h2o_hist_root16(P->fine16, P->f16_planes, P->unit ? nullptr : tp_aux(P, 0), tp_aux(P, 1), P->N, P->meta[0],
                             P->f16col, P->f16n, P->F, P->partials, P->slot, P->qs, g0, P->pf32, s));
  else
  TP_CHECK(h2o_hist_build(P->master, P->stride, P->unit ? nullptr : tp_aux(P, 0), tp_aux(P, 1), P->nodes[0], P->bp[0],
                          P->meta[0], P->F, P->partials, P->slot, P->qs, g0, P->packed, nullptr, nullptr, P->pf32, P->N,
                          P->planar | (P->no_na << 1), P->nbins_f, P->fine_f, tp_planes(tp_fcut(P, 0)), nullptr, s));
  // row-sharded all-reduce: straight into the wire buffer; sliced: hbuild (packed by slice next)
  if (P->dist && !P->sliced)
    return h2o_hist_reduce(P->partials, P->slot, P->used, P->nodes[0], P->bp[0], P->meta[0], 1, g0, P->hrecv, nullptr,
                           nullptr, P->pf32, P->cf32, P->sslot, tp_fcut(P, 0), s);
  return h2o_hist_reduce(P->partials, P->slot, P->used, P->nodes[0], P->bp[0], P->meta[0], 1, g0,
                         P->sliced ? P->hbuild : P->hist0, nullptr, nullptr, P->pf32, 0, 0,
                         tp_fcut(P, 0), s);
}

// split search of level d: every feature into cand, or (sliced) this rank's feature slice into cand_local.
// Row-sharded: the level's node histograms are derived from the exchanged build slots on the way (Derive).
int h2o_tree_find(const TreePlan* P, int d, hipStream_t s) {
  void* hc = (d % 2) ? P->hist1 : P->hist0;
  const void* hp = (d % 2) ? P->hist0 : P->hist1;      // level d-1 (unused at the root: build = 1)
  SplitParams p;
  p.min_w = P->min_w; p.min_split_improvement = P->msi; p.lambda = P->lam; p.alpha = P->alpha; p.gamma = P->gamma;
  p.mode = P->mode; p.random_split = P->random_split; p.seed = P->seed; p.hist_type = P->hist_type;
  p.fcut = tp_fcut(P, d);
  tp_node_range(P, d, hp, p);
  const int hs = P->sliced ? P->sslot : P->slot;
  const Derive dv = P->dist ? Derive{P->hrecv, P->cf32, P->sslot, (const double*)hp, (const Node*)P->nodes[d]}
                            : Derive{nullptr, 0, 0, nullptr, nullptr};
  if (!P->sliced)
    return split_find_launch(hc, hs, P->meta[d], P->caps[d], P->F, P->nbins_f, P->iscat_f, P->mono_f, p, d, P->cand,
                             d == 0 ? P->rootw : nullptr, P->edges, P->nb_level[d], 0, P->F, dv, s);
  const int f0 = P->fs0;
  return split_find_launch(hc, hs, P->meta[d], P->caps[d], P->fsn, (const int*)P->nbins_f + f0,
                           (const int*)P->iscat_f + f0, P->mono_f ? (const int*)P->mono_f + f0 : nullptr, p, d,
                           P->cand_local, d == 0 ? P->rootw : nullptr,
                           P->edges ? (const float*)P->edges + (size_t)f0 * 255 : nullptr, P->nb_level[d], f0,
                           (P->sslot - 1) / (2 * NBIN + 1), dv, s);
}

// decisions (from cand) + plan, then the next level's histogram.
// returns 0 = histogram done (dist: compact buffer ready for the collective), 1 = last level, <0 error.
static int tree_grow(const TreePlan* P, int d, int dist, hipStream_t s, bool plan_done);
int h2o_tree_grow(const TreePlan* P, int d, int dist, hipStream_t s) { return tree_grow(P, d, dist, s, false); }

// single-process levels of <= PLAN_REDUCE_MAX nodes: split search + plan in one launch (k_split_find_plan). OFF by
// default (H2O_PLAN_FUSED=1 turns it on). MEASURED r5 (scripts/gpu_r5_c15.sh, 11M HIGGS): the per-block agent-scope
// release (buffer_wbl2) of the ticket made k_split_find_plan 16-43 us per level against 13-19 for the two launches,
// and the tree 1.262 -> 1.372 ms (24 dispatches instead of 31): on MI355X an L2 write-back per block costs far more
// than a kernel boundary.
static bool plan_fused() {
  static int v = -1;
  if (v < 0) { const char* e = getenv("H2O_PLAN_FUSED"); v = (e && e[0] == '1') ? 1 : 0; }
  return v == 1;
}

static int tree_find_plan(const TreePlan* P, int d, hipStream_t s) {
  void* hc = (d % 2) ? P->hist1 : P->hist0;
  SplitParams p;
  p.min_w = P->min_w; p.min_split_improvement = P->msi; p.lambda = P->lam; p.alpha = P->alpha; p.gamma = P->gamma;
  p.mode = P->mode; p.random_split = P->random_split; p.seed = P->seed; p.hist_type = P->hist_type;
  p.fcut = tp_fcut(P, d);
  tp_node_range(P, d, (d % 2) ? P->hist0 : P->hist1, p);
  const int cap = P->caps[d];
  const int kc = P->kc_level[d] > 0 ? P->kc_level[d] : P->k_cols;
  const PlanReduce pr{(const Cand*)P->cand, P->F, (const int*)P->feat_ok, kc, P->seed,
                      P->ic_map ? (const unsigned char*)P->ic[d] : nullptr, (const int*)P->fgroup, 0, cap};
  const bool odd = d % 2 == 1;
  const PlanArgs pa{(const Node*)P->nodes[d], (const int*)P->meta[d], (Dec*)P->dec[d], (int*)P->nl[d],
                    odd ? (const int*)P->nl[d - 1] : nullptr, (int4*)P->cur[d], (int*)P->cl[d], (int*)P->cr[d],
                    (Node*)P->nodes[d + 1], (int*)P->tp[d + 1], (int*)P->meta[d + 1], (int*)P->bp[d + 1],
                    (int*)P->counters, (int*)P->scratch, d, P->D, P->caps[d + 1], P->leaf_cap, P->min_w, pr,
                    (int*)P->counters + 2};
  if (P->F <= 0 || cap <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_split_find_plan, dim3(cap, P->F), dim3(256), 0, s, (double*)hc, P->slot, (const int*)P->meta[d],
                     P->F, (const int*)P->nbins_f, (const int*)P->iscat_f, (const int*)P->mono_f, p, d,
                     (Cand*)P->cand, d == 0 ? (double*)P->rootw : nullptr, (const float*)P->edges, P->nb_level[d], 0,
                     P->F, Derive{nullptr, 0, 0, nullptr, nullptr}, pa);
  return (int)hipGetLastError();
}

static int tree_grow(const TreePlan* P, int d, int dist, hipStream_t s, bool plan_done) {
  void* hc = (d % 2) ? P->hist1 : P->hist0;
  void* hn = (d % 2) ? P->hist0 : P->hist1;
  const int cap = P->caps[d];
  const bool odd = d % 2 == 1;
  int rc;
  const int kc = P->kc_level[d] > 0 ? P->kc_level[d] : P->k_cols;
  // small levels: the plan block picks the decisions itself (one launch instead of two)
  // sliced: the rank-major all-gather of every rank's candidates, read in place (cand_at)
  const void* cand = P->sliced ? P->cand_all : P->cand;
  const int cfs = P->sliced ? P->cand_fs : 0;
  PlanReduce pr{nullptr, P->F, (const int*)P->feat_ok, kc, P->seed,
                P->ic_map ? (const unsigned char*)P->ic[d] : nullptr, (const int*)P->fgroup, cfs, cap};
  if (!plan_done) {
    if (cap <= PLAN_REDUCE_MAX) {
      pr.cand = (const Cand*)cand;
    } else {
      rc = h2o_split_reduce(cand, P->meta[d], cap, P->F, P->feat_ok, kc, P->seed, d, P->dec[d],
                            P->ic_map ? P->ic[d] : nullptr, P->fgroup, cfs, s);
      if (rc) return -rc;
    }
    rc = plan_launch(P->nodes[d], P->meta[d], P->dec[d], P->nl[d], odd ? P->nl[d - 1] : nullptr, P->cur[d], P->cl[d],
                     P->cr[d], P->nodes[d + 1], P->tp[d + 1], P->meta[d + 1], P->bp[d + 1], P->counters, P->scratch,
                     d, P->D, P->min_w, P->caps[d + 1], P->leaf_cap, pr, s);
    if (rc) return -rc;
  }
  if (P->ic_map && d + 1 < P->D) {
    rc = h2o_ic_next(P->nodes[d + 1], P->meta[d + 1], P->dec[d], P->ic[d], P->ic_map, P->F, P->ic[d + 1],
                     P->caps[d + 1], s);
    if (rc) return -rc;
  }
  if (d + 1 == P->D) return 1;             // every row's leaf: h2o_tree_leaves over the original order
  int gh;
  const void *sb, *sy, *sw;
  if (!odd) {
    // level d+1 (odd) is histogrammed straight from level d's ranges, filtered by level d's decisions
    gh = P->tiles_cap[d] < P->grid ? P->tiles_cap[d] : P->grid;
    tp_level_buf(P, d, sb, sy, sw);
    // level 1 of a narrow planar run: the root split's side of every row as bytes (read by the level-1
    // histogram blocks and the root route instead of the split column's plane)
    const void* fdir = nullptr;
    // (also every planar run whose level 1 builds >= 2 planes, e.g. XGBoost 100M x 50: each plane's histogram blocks
    // would otherwise read the root split column's plane once per plane)
    if (d == 0 && P->fdir && (tp_lvl2(P) || (P->planar && tp_planes(tp_fcut(P, 1) > 0 ? tp_fcut(P, 1) : P->F) >= 2))) {
      long long g = (P->N + 255) / 256;
      if (g > 4096) g = 4096;
      if (g < 1) g = 1;
      hipLaunchKernelGGL(k_row_dir, dim3((unsigned)g), dim3(256), 0, s, (const uint8_t*)P->master, P->stride, P->N,
                         P->planar, (const Dec*)P->dec[0], (uint8_t*)P->fdir);
      rc = (int)hipGetLastError();
      if (rc) return -rc;
      fdir = P->fdir;
    }
    rc = h2o_hist_build(sb, P->stride, sw, sy, P->nodes[d + 1], P->bp[d + 1], P->meta[d + 1], P->F, P->partials,
                        P->slot, P->qs, gh, P->packed, P->dec[d], P->nl[d], P->pf32, P->N, P->planar | (P->no_na << 1),
                        P->nbins_f, P->fine_f, tp_planes(tp_fcut(P, d + 1)), fdir, s);
  } else {
    // regroup level d-1's rows two levels down, then histogram level d+1 (even) contiguously
    const bool fused = route_fused_ranges() && P->tiles_cap[d - 1] > 0;
    rc = tp_route(P, d - 1, s, fused);
    if (rc) return -rc;
    if (!fused) {
      rc = h2o_ranges(P->nodes[d + 1], P->cur[d], P->tp[d + 1], P->bp[d + 1], P->meta[d + 1], s);
      if (rc) return -rc;
    }
    gh = P->tiles_cap[d + 1] < P->grid ? P->tiles_cap[d + 1] : P->grid;
    tp_level_buf(P, d + 1, sb, sy, sw);
    rc = h2o_hist_build(sb, P->stride, sw, sy, P->nodes[d + 1], P->bp[d + 1], P->meta[d + 1], P->F, P->partials,
                        P->slot, P->qs, gh, P->packed, nullptr, nullptr, P->pf32, P->N, P->planar | (P->no_na << 1),
                        P->nbins_f, P->fine_f, tp_planes(tp_fcut(P, d + 1)), nullptr, s);
  }
  if (rc) return -rc;
  const int lo = tp_fcut(P, d + 1);
  if (!dist)
    rc = h2o_hist_reduce(P->partials, P->slot, P->used, P->nodes[d + 1], P->bp[d + 1], P->meta[d + 1], P->caps[d + 1],
                         gh, nullptr, hn, hc, P->pf32, 0, 0, lo, s);
  else if (P->sliced)
    rc = h2o_hist_reduce(P->partials, P->slot, P->used, P->nodes[d + 1], P->bp[d + 1], P->meta[d + 1], P->caps[d + 1],
                         gh, P->hbuild, nullptr, nullptr, P->pf32, 0, 0, lo, s);
  else   // all-reduce exchange: the build slots go straight into the wire buffer
    rc = h2o_hist_reduce(P->partials, P->slot, P->used, P->nodes[d + 1], P->bp[d + 1], P->meta[d + 1], P->caps[d + 1],
                         gh, P->hrecv, nullptr, nullptr, P->pf32, P->cf32, P->sslot, lo, s);
  return rc ? -rc : 0;
}

// one level: split search, decisions, plan, next histogram (single process and all-reduce mode)
int h2o_tree_level(const TreePlan* P, int d, int dist, hipStream_t s) {
  const bool fuse = !dist && !P->dist && !P->sliced && P->caps[d] <= PLAN_REDUCE_MAX && plan_fused() && !P->gcat;
  const int rc = fuse ? tree_find_plan(P, d, s) : h2o_tree_find(P, d, s);
  if (rc) return -rc;
  return tree_grow(P, d, dist, s, fuse);
}


// after the last level: leaf_of_row (original order) + fp64 leaf sums (the caller all-reduces them when sharded)
static int tree_leaves(const TreePlan* P, bool values, hipStream_t s) {
  int n_nodes = 0;
  for (int d = 0; d < P->D; ++d) n_nodes += P->caps[d];
  const LeafVals lv{P->log_link, P->scale, P->kclamp, P->mx, P->leaf_lam, P->leaf_l1,
                    values ? (float*)P->leafval : nullptr};
  // (H2O_LEAF_FUSED=1: k_leafsum_finish in the leaf-assign launch's last block. OFF by default — MEASURED r5: the
  // 2048 per-block release fences made k_leaf_assign 221 us against 115 + 4 for the two launches)
  static int fused = -1;
  if (fused < 0) { const char* e = getenv("H2O_LEAF_FUSED"); fused = (e && e[0] == '1') ? 1 : 0; }
  return leaf_assign_launch(P->master, P->stride, P->N, P->lvptrs, P->D, tp_aux(P, P->num_plane), tp_aux(P, 3), P->qs,
                            P->leaf_of_row, P->leafq, P->leaf_cap, P->leafsum, n_nodes, P->planar, lv, s, tp_lvl2(P),
                            fused ? (int*)P->counters + 3 : nullptr, P->gcat != nullptr);
}

int h2o_tree_leaves(const TreePlan* P, hipStream_t s) { return tree_leaves(P, false, s); }

static inline int coll(const TreePlan* P, int op, const void* snd, void* rcv, long long count, int dt, hipStream_t s) {
  return ((h2o_coll_fn)P->coll_fn)(P->coll_ctx, op, snd, rcv, count, dt, s);
}

// The histogram exchange of n build slots (src: slots of `slot` doubles, slot = parent) into hrecv, in the wire
// dtype (cf32: fp32, half the bytes; else fp64):
//  * sliced: pack by feature slice into hsend [W][n][sslot] and REDUCE-SCATTER -> hrecv [n][sslot] holds the
//    GLOBAL histograms of this rank's features;
//  * all-reduce: k_hist_reduce wrote the build slots straight into hrecv ([n][E = used]); ALL-REDUCE in place.
// The next k_split_find derives the node histograms from hrecv (fused sibling subtraction).
static int exchange(const TreePlan* P, int n, hipStream_t s) {
  const int dt = P->cf32 ? H2O_DT_F32 : H2O_DT_F64;
  if (P->sliced) {
    TP_CHECK(h2o_hist_pack(P->hbuild, P->slot, P->F, P->cand_fs, P->W, n, P->hsend, P->cf32, s));
    return coll(P, H2O_COLL_REDUCE_SCATTER, P->hsend, P->hrecv, (long long)n * P->sslot, dt, s);
  }
  // k_hist_reduce already wrote the build slots into hrecv ([n][E = used], wire dtype)
  return coll(P, H2O_COLL_ALLREDUCE, P->hrecv, P->hrecv, (long long)n * P->sslot, dt, s);
}

// Row-sharded tree (reference: hex/tree/ScoreBuildHistogram2.java + water/MRTask.java reduce), the whole tree
// in ONE host call: every kernel and every collective is enqueued on stream s in order, the host never waits.
//  * all-reduce (default): per level the built-node histograms are all-reduced; every rank searches every
//    feature of the same global histograms, so every rank takes the same decisions. One collective per level.
//  * sliced: per level the built-node histograms are reduce-scattered by feature slice (rank r gets the GLOBAL
//    histograms of features [r*Fs, r*Fs+Fs)), each rank searches its slice, and the per-(node, feature)
//    candidates are all-gathered (a few KB, read in place rank-major): 1/W of the split search per rank, but two
//    collectives per level.
// Both end with one all-reduce of the leaf sums (sliced: + the root weight, which only the owner of feature 0
// computes).
int h2o_tree_dist(const TreePlan* P, hipStream_t s) {
  if (!P->coll_fn || P->W < 1) return (int)hipErrorInvalidValue;
  if (!P->dist) return (int)hipErrorInvalidValue;
  TP_CHECK(h2o_tree_root(P, s));               // -> hbuild slot 0 (sliced) / hrecv slot 0
  const long long L2 = 2LL * P->leaf_cap;
  TP_CHECK(exchange(P, 1, s));
  for (int d = 0; d < P->D; ++d) {
    TP_CHECK(h2o_tree_find(P, d, s));
    if (P->sliced)
      TP_CHECK(coll(P, H2O_COLL_ALLGATHER, P->cand_local, P->cand_all,
                    (long long)P->caps[d] * P->cand_fs * (long long)sizeof(Cand), H2O_DT_U8, s));
    const int r = h2o_tree_grow(P, d, 1, s);
    if (r < 0) return -r;
    if (r == 1) break;
    TP_CHECK(exchange(P, P->caps[d], s));
  }
  TP_CHECK(h2o_tree_leaves(P, s));
  if (P->sliced) {
    double* lsx = (double*)P->lsx;
    TP_CHECK((int)hipMemcpyAsync(lsx, P->leafsum, (size_t)L2 * 8, hipMemcpyDeviceToDevice, s));
    if (P->fs0 == 0 && P->fsn > 0)
      TP_CHECK((int)hipMemcpyAsync(lsx + L2, P->rootw, 8, hipMemcpyDeviceToDevice, s));
    else
      TP_CHECK((int)hipMemsetAsync(lsx + L2, 0, 8, s));
    TP_CHECK(coll(P, H2O_COLL_ALLREDUCE, lsx, lsx, L2 + 1, H2O_DT_F64, s));
    TP_CHECK((int)hipMemcpyAsync(P->leafsum, lsx, (size_t)L2 * 8, hipMemcpyDeviceToDevice, s));
    TP_CHECK((int)hipMemcpyAsync(P->rootw, lsx + L2, 8, hipMemcpyDeviceToDevice, s));
  } else {
    TP_CHECK(coll(P, H2O_COLL_ALLREDUCE, P->leafsum, P->leafsum, L2, H2O_DT_F64, s));
  }
  if (P->leaf_native)
    TP_CHECK(h2o_leaf_values(P->leafsum, P->leaf_cap, P->log_link, P->scale, P->kclamp, P->mx, P->leaf_lam,
                             P->leaf_l1, P->leafval, s));
  return 0;
}

// single process: the whole tree (root .. leaves, and leaf_native values in the leaf-sum pass) in one host call
int h2o_tree_all(const TreePlan* P, hipStream_t s) {
  TP_CHECK(h2o_tree_root(P, s));
  for (int d = 0; d < P->D; ++d) {
    const int r = h2o_tree_level(P, d, 0, s);
    if (r < 0) return -r;
    if (r == 1) break;
  }
  return tree_leaves(P, P->leaf_native != 0, s);
}
#undef TP_CHECK

}  // extern "C"
