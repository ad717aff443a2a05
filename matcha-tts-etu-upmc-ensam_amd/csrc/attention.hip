// Flash attention (forward + deterministic backward) for the decoder's transformer blocks on gfx950
// MFMA.  Reference: transformer.py:191-370 (diffusers Attention, 4 heads x 64; head dims 32/64/96
// are built) whose mask reaches
// F.scaled_dot_product_attention as a FLOAT tensor, i.e. an additive per-key bias (the 0/1 mask
// itself: +1 on valid keys, +0 on padding -- padded keys are NOT excluded).  scores = q.k*scale + bias.
//
// Layout: q/k/v/o and their gradients are token-major rows (row = b*T + t) with head h at columns
// [h*64, h*64+64) -- the fused QKV projection's output is consumed in place, no transposes.
//
// Orientation trick.  A 32x32 MFMA tile's C layout gives lane l the column (l & 31) and 16 rows
// {(v&3) + 8(v>>2) + 4(l>>5)}.  The forward and dQ kernels compute S^T = K Q^T, so a lane owns ONE
// query and 16 keys of the tile (its partner lane l^32 the other 16): the row softmax is 16 in-lane
// values + one lane^32 exchange, the online-softmax rescale is a per-lane scalar, and P^T feeds the
// next MFMA (O^T += V^T P^T) straight from registers because the V^T fragment is read from LDS in the
// same key order the lane holds.  The dK/dV kernel uses the mirrored orientation (a lane owns one key).
// Softmax runs in the log2 domain; the saved row statistic is lse2 = log2(sum_j 2^(s2_ij)).
//
// Precision: BF16 = bf16 MFMA (32x32x16) operands, fp32 accumulation and softmax (bf16-mixed mode);
// FP32 = exact-fp32 MFMA (32x32x2) -- the parity mode.  Inputs/outputs are fp32 in HBM either way.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <type_traits>

#include "mtts_common.h"
#include "mtts_decoder.h"

namespace {
// XCD-aware block order (round 4): the dispatcher deals the linear block id (x fastest, then y, then z) round
// robin over the 8 XCDs, so the query blocks of one (b, h) pair landed on 8 different L2s, each fetching that
// pair's K / V (PMC: 1.78x the algorithmic bytes).  The id is relabelled so that consecutive (x, y, z) -- every
// block of one pair, and for the merged backward both its dQ and dK / dV halves -- run on one XCD (the same
// bijection as mtts::xcd_relabel of the GEMMs).
__device__ __forceinline__ int3 xcd_blk3() {
    const int gx = (int)gridDim.x, gy = (int)gridDim.y, nwg = gx * gy * (int)gridDim.z;
    const int orig = (int)blockIdx.x + gx * ((int)blockIdx.y + gy * (int)blockIdx.z);
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    const int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
    const int x = w % gx, t = w / gx;
    return make_int3(x, t % gy, t / gy);
}
}  // namespace

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kTile = 64;           // keys (fwd, dQ) or queries (dKV) per LDS stage
constexpr int kRowsPerBlock = 128;  // queries (fwd, dQ) or keys (dKV) per block: 4 waves x 32
constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr float kLog2e = 1.4426950408889634f;
constexpr size_t kLdsMax = 160 * 1024;

// Geometry per (precision, compiled head dim D in {32, 64, 96}; a runtime head dim dh <= D runs with
// zero-filled columns dh..D-1).  Row tiles are [64 rows][D + pad] (fragment
// reads along the head dim), transposed tiles [D][64 + pad] (fragment reads along the rows).
//
// bf16: ONE swizzled image per tile, read by rows (ds_read_b128) for the MFMAs that sum over the head
// dim and by columns (ds_read_b64_tr_b16, the gfx950 transposing LDS read) for the MFMAs that sum over
// the tile's rows -- no transposed copy, every store a ds_write_b64.  The image is made of 8-row x
// 32-column sub-tiles of 512 B ([row / 8][col / 32][row % 8][32 cols]); inside a sub-tile row the
// 16-byte chunk ch sits at chunk ch ^ ((row >> 2) & 3).  With the staging map below (16 lanes = two
// rows x 32 columns) the b64 stores, the b128 row reads and the transposing reads of the 32x32x16
// operand maps are all bank-conflict free (checked exhaustively for D = 32 / 64 / 96 against the
// lane groups of MI355X_MICROARCH.md's LDS table), and the per-lane read addresses differ only by
// immediates across k-steps / sub-tiles but for the XOR's one varying bit (2 base registers each).
// fp32 (parity mode): a padded row tile plus a transposed tile, scalar fragment reads.
template <bool BF16, int D>
struct G {
    static_assert(D % 32 == 0 && D <= 96, "head dim 32, 64 or 96");
    using T = std::conditional_t<BF16, uint16_t, float>;
    static constexpr int LDR = D + 1;               // fp32 row tile pitch (elements)
    static constexpr int LDT = kTile + 1;           // fp32 transposed tile pitch
    static constexpr int RE = BF16 ? kTile * D : kTile * LDR;  // elements of a row tile / image
    static constexpr int TE = BF16 ? 0 : D * LDT;   // elements of a transposed tile (fp32 only)
    static constexpr int NT = D / 32;               // 32-wide MFMA tiles over the head dim
    static constexpr int F4 = kTile * D / 4 / kThreads;  // float4 per thread to stage one tile
};

// byte offset of elements (r, col .. col+3) in a bf16 image (col % 4 == 0)
template <int D>
__device__ __forceinline__ int img_off(int r, int col) {
    return 16 * D * (r >> 3) + 512 * (col >> 5) + 64 * (r & 7) + 16 * (((col >> 3) & 3) ^ ((r >> 2) & 3)) +
           8 * ((col >> 2) & 1);
}

// staging map of float4 number idx of a 64 x D tile: fp32 row-major; bf16 16-lane groups of two rows
// x 32 columns (one 128-byte span of the image per group: conflict-free b64 stores)
template <bool BF16, int D>
__device__ __forceinline__ void stage_rc(int idx, int &r, int &c) {
    if constexpr (BF16) {
        constexpr int NT = D / 32;
        const int cc = idx & 7, rr = (idx >> 3) & 1, g = idx >> 4;
        r = 2 * (g / NT) + rr;
        c = 32 * (g % NT) + 4 * cc;
    } else {
        r = idx / (D / 4);
        c = (idx % (D / 4)) * 4;
    }
}

typedef short v4i16 __attribute__((ext_vector_type(4)));
// ds_read_b64_tr_b16: in each 16-lane group, lane 4q+p addresses row q / columns 4p..4p+3 of a 4x16
// block and lane i receives column i of the 4 rows (EXEC must be full: called outside divergence)
__device__ __forceinline__ uint2 lds_tr16(const void *p) {
    const v4i16 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4i16 *)(const_cast<void *>(p)));
    return __builtin_bit_cast(uint2, v);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// (a, b) -> one v_cvt_pk_bf16_f32 (two scalar conversions + shift/or compile to 4 instructions)
__device__ __forceinline__ uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}
// bf16 fragments are always assembled from 32-bit words: element-wise construction of bf16 / u16
// vectors from LDS loads miscompiles here (every element comes back as element 0), like the
// raw_buffer_load_b64 builtin (toolchain findings).
__device__ __forceinline__ bf16x8 frag8(const float *e) {
    const uint4 w = make_uint4(pack2(e[0], e[1]), pack2(e[2], e[3]), pack2(e[4], e[5]), pack2(e[6], e[7]));
    return __builtin_bit_cast(bf16x8, w);
}

__device__ __forceinline__ int crow(int v, int lh) { return (v & 3) + 8 * (v >> 2) + 4 * lh; }

// q / k / v / o / dO / dq / dk / dv storage (TI): fp32, or bf16 bits (uint16_t, MTTS_ATTN_F_IO_BF16 in
// bf16-mixed mode: the MFMA operands are bf16 anyway, so the producers' GEMMs write half the bytes)
template <typename TI>
__device__ __forceinline__ float4 ld4f(const TI *p) {
    if constexpr (sizeof(TI) == 4) {
        return *reinterpret_cast<const float4 *>(p);
    } else {
        const uint2 q = *reinterpret_cast<const uint2 *>(p);
        return make_float4(__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u),
                           __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u));
    }
}
template <typename TI>
__device__ __forceinline__ void st4f(TI *p, float4 v) {
    if constexpr (sizeof(TI) == 4) *reinterpret_cast<float4 *>(p) = v;
    else *reinterpret_cast<uint2 *>(p) = make_uint2(pack2(v.x, v.y), pack2(v.z, v.w));
}

// The 16 C-layout rows a lane holds are 4 runs of 4: per-row LDS constants (key bias, lse, D) are
// read as 4 float4 (ds_read_b128) instead of 16 scalars.
__device__ __forceinline__ void crow_load16(const float *base, int lh, float (&out)[16]) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const float4 t = *reinterpret_cast<const float4 *>(base + 8 * g + 4 * lh);
        out[4 * g] = t.x;
        out[4 * g + 1] = t.y;
        out[4 * g + 2] = t.z;
        out[4 * g + 3] = t.w;
    }
}

// x combined with the other 32-lane half's value of the same lane slot (v_permlane32_swap: no LDS)
__device__ __forceinline__ float half_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float half_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// 2^x as the bare v_exp_f32: arguments are <= kDefer or -inf (-> 0); tiny results flush to zero
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// B-operand fragments held in registers for one row (a query or a key) of the lane: the row's D
// dims in MFMA k-step order.
template <bool BF16, int D>
struct RowFrag;
template <int D>
struct RowFrag<true, D> {
    bf16x8 f[D / 16];
    // mul: a prescale folded into the operand before its bf16 rounding (the softmax scale * log2 e)
    template <typename TI>
    __device__ void load(const TI *row, bool ok, int lh, int dh, float mul = 1.f) {
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) {
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
            const int c = 16 * ks + 8 * lh;
            if (ok && c < dh) a = ld4f(row + c);
            if (ok && c + 4 < dh) b = ld4f(row + c + 4);
            const float e[8] = {a.x * mul, a.y * mul, a.z * mul, a.w * mul,
                                b.x * mul, b.y * mul, b.z * mul, b.w * mul};
            f[ks] = frag8(e);
        }
    }
};
template <int D>
struct RowFrag<false, D> {
    float f[D / 2];
    __device__ void load(const float *row, bool ok, int lh, int dh, float = 1.f) {
#pragma unroll
        for (int ks = 0; ks < D / 2; ++ks) f[ks] = (ok && 2 * ks + lh < dh) ? row[2 * ks + lh] : 0.f;
    }
};

// acc += A(LDS row tile, row r, contiguous over the head dim) x B(register row fragment)
template <bool BF16, int D>
__device__ __forceinline__ void mma_rows(f32x16 &acc, const typename G<BF16, D>::T *tile, int r, int lh,
                                         const RowFrag<BF16, D> &bf) {
    constexpr int LD = G<BF16, D>::LDR;
    if constexpr (BF16) {
        const char *img = reinterpret_cast<const char *>(tile);
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) {
            const bf16x8 a = *reinterpret_cast<const bf16x8 *>(img + img_off<D>(r, 16 * ks + 8 * lh));
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bf.f[ks], acc, 0, 0, 0);
        }
    } else {
#pragma unroll
        for (int ks = 0; ks < D / 2; ++ks)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(tile[r * LD + 2 * ks + lh], bf.f[ks], acc, 0, 0, 0);
    }
}

// acc += A(the tile transposed: row = head dim d, columns = the 32 rows of sub-tile `sub`, read in
// the C-layout order this lane holds) x B(the lane's 16 C-layout values `s`).  bf16: `tileT` is the
// row image, read with the transposing LDS read; fp32: the transposed tile.
template <bool BF16, int D>
__device__ __forceinline__ void mma_perm(f32x16 &acc, const typename G<BF16, D>::T *tileT, int d, int sub, int lh,
                                         const float (&s)[16]) {
    constexpr int LD = G<BF16, D>::LDT;
    if constexpr (BF16) {
        // lane's k-slots = rows {16ks + 4lh + 0..3, 16ks + 8 + 4lh + 0..3} of the sub-tile (the C-layout
        // rows it holds in s[8ks .. 8ks+7]); group lane 4q+p addresses row q, columns 4p.. of its block
        const char *img = reinterpret_cast<const char *>(tileT);
        const int j = threadIdx.x & 15, g1 = (threadIdx.x >> 4) & 1;
        const int col = (d & ~31) + 16 * g1 + 4 * (j & 3);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int r = sub * 32 + 16 * ks + 4 * lh + (j >> 2);
            const uint2 lo = lds_tr16(img + img_off<D>(r, col));
            const uint2 hi = lds_tr16(img + img_off<D>(r + 8, col));
            const bf16x8 a = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
            const bf16x8 b = frag8(s + 8 * ks);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
        }
    } else {
#pragma unroll
        for (int v = 0; v < 16; ++v)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(tileT[d * LD + sub * 32 + crow(v, lh)], s[v], acc, 0, 0, 0);
    }
}

// Staging of a 64-row tile of one head (rows r0.. of batch b) into LDS: row layout and/or transposed.
// TI = uint16_t (bf16 storage, bf16 MFMA): the 4 bf16 of a chunk travel as raw bits into the image --
// no unpack to fp32 and repack.
template <bool BF16, int D, typename TI = float>
struct TileLoader {
    using Gm = G<BF16, D>;
    static constexpr bool kRaw = BF16 && sizeof(TI) == 2;
    float4 v[kRaw ? 1 : Gm::F4];
    uint2 r[kRaw ? Gm::F4 : 1];
    bool narrow = false;  // runtime head dim dh < D: columns past dh are zeroed
    // unconditional loads from clamped addresses: no branch around a load, so the loads stay in flight
    // through the compute phase.  Rows past T are NOT zeroed: they hold finite data (row 0 of the
    // batch) and every kernel gives them probability 0 (key bias -inf / query lse +inf), so they add
    // exact zeros to every product.
    __device__ void load(const TI *base, int ld, int b, int T, int r0, int tid, int dh) {
        narrow = dh < D;
        const TI *bb = base + (size_t)b * T * ld;  // batch b, row 0
#pragma unroll
        for (int i = 0; i < Gm::F4; ++i) {
            int rr, c;
            stage_rc<BF16, D>(tid + kThreads * i, rr, c);
            const bool ok = r0 + rr < T && c < dh;
            const TI *src = bb + (ok ? (r0 + rr) * ld + c : 0);
            if constexpr (kRaw) r[i] = *reinterpret_cast<const uint2 *>(src);
            else v[i] = ld4f(src);
        }
    }
    __device__ void store(typename Gm::T *rowt, typename Gm::T *trt, int tid, int dh) const {
#pragma unroll
        for (int i = 0; i < Gm::F4; ++i) {
            int rr, c;
            stage_rc<BF16, D>(tid + kThreads * i, rr, c);
            if constexpr (kRaw) {
                uint2 w = r[i];
                if (narrow && c >= dh) w = make_uint2(0u, 0u);
                typename Gm::T *img = rowt ? rowt : trt;
                if (img) *reinterpret_cast<uint2 *>(reinterpret_cast<char *>(img) + img_off<D>(rr, c)) = w;
                continue;
            } else {
                float e[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
                if (narrow && c >= dh) e[0] = e[1] = e[2] = e[3] = 0.f;
                if constexpr (BF16) {  // one image serves both reads: `trt` names it when `rowt` is null
                    typename Gm::T *img = rowt ? rowt : trt;
                    if (img)
                        *reinterpret_cast<uint2 *>(reinterpret_cast<char *>(img) + img_off<D>(rr, c)) =
                            make_uint2(pack2(e[0], e[1]), pack2(e[2], e[3]));
                } else {
                    if (rowt) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) rowt[rr * Gm::LDR + c + j] = e[j];
                    }
                    if (trt) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) trt[(c + j) * Gm::LDT + rr] = e[j];
                    }
                }
            }
        }
    }
};

// LDS bytes per stage; kernels double-buffer when two stages fit in 160 KB, else single-buffer.
template <bool BF16, int D>
constexpr size_t fwd_stage() {  // K rows + V transposed (bf16: K and V images) + bias
    return (size_t)(G<BF16, D>::RE + (BF16 ? G<BF16, D>::RE : G<BF16, D>::TE)) * sizeof(typename G<BF16, D>::T) +
           kTile * sizeof(float);
}
template <bool BF16, int D>
constexpr size_t dq_stage() {  // K rows + V rows + K transposed + bias
    return (size_t)(2 * G<BF16, D>::RE + G<BF16, D>::TE) * sizeof(typename G<BF16, D>::T) + kTile * sizeof(float);
}
template <bool BF16, int D>
constexpr size_t dkv_stage() {  // Q rows + dO rows + Q transposed + dO transposed + lse + Drow
    return (size_t)(2 * G<BF16, D>::RE + 2 * G<BF16, D>::TE) * sizeof(typename G<BF16, D>::T) +
           2 * kTile * sizeof(float);
}
constexpr int nbuf(size_t stage) { return 2 * stage <= kLdsMax ? 2 : 1; }

template <typename T>
__device__ __forceinline__ T *carve(unsigned char *&p, size_t n) {
    T *r = reinterpret_cast<T *>(p);
    p += (n * sizeof(T) + 15) / 16 * 16;
    return r;
}

// The key bias enters shifted by the batch row's first bias c0 -- softmax is invariant to a per-row
// constant, and the saved lse carries the shift consistently into the backward.  With the 0/1 key mask
// every tile inside the valid keys is then all zeros: the stage's flag lets it skip the per-element
// bias (wave 0 stages the 64 biases of a tile and votes).
__device__ __forceinline__ float key_bias_c0(const mtts_attn_args &p, int b) {
    return p.key_bias ? p.key_bias[(size_t)b * p.T] : 0.f;
}
__device__ __forceinline__ float stage_bias(const mtts_attn_args &p, int b, int key, float c0) {
    const int T = p.T;
    const float raw = *(p.key_bias ? p.key_bias + (size_t)b * T + min(key, T - 1) : p.q);
    return key < T ? (p.key_bias ? (raw - c0) * kLog2e : 0.f) : -INFINITY;
}
__device__ __forceinline__ void store_bias(float *bias_s, int *flag_s, int buf, float bias_r, int tid) {
    if (tid < kTile) {  // wave 0, all lanes
        bias_s[buf * kTile + tid] = bias_r;
        const bool nz = __any(bias_r != 0.f);
        if (tid == 0) flag_s[buf] = nz;
    }
}

// Online-softmax rescales are deferred while the running max grows by at most kDefer (log2 units):
// the probabilities then stay <= 2^kDefer, exact in fp32 and harmless to bf16 (the normaliser l uses
// the same stale max).  The decision is wave-uniform, so the 16 x NT accumulator multiplies are
// skipped as a whole on most tiles.
constexpr float kDefer = 8.f;

// The shared K-tile loop: stage 0, then per tile prefetch the next into registers, compute, and
// publish it (double buffer: into the other stage, one barrier; single buffer: two barriers).
template <int NB, typename Load, typename Store, typename Compute>
__device__ __forceinline__ void tile_loop(int ntiles, Load &&load, Store &&store, Compute &&compute) {
    // LDS-only barriers (mtts::lds_barrier): the next tile's global loads stay in flight across them
    load(0);
    store(0);
    mtts::lds_barrier();
    for (int it = 0; it < ntiles; ++it) {
        const int buf = NB == 2 ? (it & 1) : 0;
        load((it + 1) * kTile);  // past the last tile every row is masked off (branch-free body)
        compute(buf, it * kTile);
        if constexpr (NB == 2) {
            store(buf ^ 1);
            mtts::lds_barrier();
        } else {
            mtts::lds_barrier();
            if (it + 1 < ntiles) {
                store(0);
                mtts::lds_barrier();
            }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// forward: grid (ceil(T/128), H, B); lane = query
// three workgroups per CU for the decoder's instance (bf16 storage, no dropout: 165 VGPRs): its 640
// workgroups at B = 32, T = 600 then run in one round instead of 512 + 128
template <bool BF16, int D, typename TI, bool DROP>
constexpr int fwd_min_blocks() { return (BF16 && D <= 64) ? ((!DROP && sizeof(TI) == 2) ? 3 : 2) : 1; }

template <bool BF16, int D, typename TI = float, bool DROP = true>
__global__ __launch_bounds__(kThreads, (fwd_min_blocks<BF16, D, TI, DROP>())) void attn_fwd_kernel(mtts_attn_args p) {
    const TI *Qp = reinterpret_cast<const TI *>(p.q), *Kp = reinterpret_cast<const TI *>(p.k),
             *Vp = reinterpret_cast<const TI *>(p.v);
    TI *Op = reinterpret_cast<TI *>(p.o);
    using Gm = G<BF16, D>;
    using ST = typename Gm::T;
    constexpr int NB = nbuf(fwd_stage<BF16, D>());
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char *sp = smem;
    ST *Ks = carve<ST>(sp, NB * Gm::RE);  // [NB][64 keys][LDR] (bf16: image)
    ST *Vt = carve<ST>(sp, NB * (BF16 ? Gm::RE : Gm::TE));  // [NB][D][LDT] V transposed (bf16: V image)
    float *bias_s = carve<float>(sp, NB * kTile);  // log2 domain, shifted by c0; -inf past T
    int *flag_s = carve<int>(sp, NB);              // stage has a nonzero bias

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int3 bk_ = xcd_blk3();
    const int b = bk_.z, h = bk_.y, T = p.T, dh = p.D;  // dh <= D: columns past dh are zero
    const int q = bk_.x * kRowsPerBlock + wave * 32 + lr;
    const bool q_ok = q < T;
    const TI *Kb = Kp + h * dh, *Vb = Vp + h * dh;
    const float c0 = key_bias_c0(p, b);

    // bf16: q carries scale * log2 e (scores come out of the MFMA in the log2 domain)
    const float sl2 = p.scale * kLog2e;
    RowFrag<BF16, D> qf;
    qf.load(Qp + h * dh + ((size_t)b * T + (q_ok ? q : 0)) * p.ldq, q_ok, lh, dh, BF16 ? sl2 : 1.f);

    f32x16 acc[Gm::NT];
#pragma unroll
    for (int t = 0; t < Gm::NT; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[t][v] = 0.f;
    float m = -INFINITY, l = 0.f;

    TileLoader<BF16, D, TI> lk, lv;
    float bias_r = 0.f;
    auto load = [&](int k0) __attribute__((always_inline)) {
        lk.load(Kb, p.ldq, b, T, k0, tid, dh);
        lv.load(Vb, p.ldq, b, T, k0, tid, dh);
        bias_r = stage_bias(p, b, k0 + (tid & (kTile - 1)), c0);
    };
    auto store = [&](int buf) __attribute__((always_inline)) {
        lk.store(Ks + buf * Gm::RE, nullptr, tid, dh);
        lv.store(nullptr, Vt + buf * (BF16 ? Gm::RE : Gm::TE), tid, dh);
        store_bias(bias_s, flag_s, buf, bias_r, tid);
    };
    const bool drop = DROP && p.dropout_p > 0.f;  // DROP = false: no dropout code
    uint32_t s0 = 0, s1 = 0;
    if (drop) {
        s0 = p.seed[0];
        s1 = p.seed[1];
    }
    const float inv_keep = mtts::dropout_scale(p.dropout_p);
    const uint32_t prow = (uint32_t)(((size_t)b * p.H + h) * T + q);  // dropout row key of this query
    auto body = [&](int buf, int k0, auto has_bias) __attribute__((always_inline)) {
        constexpr bool TB = decltype(has_bias)::value;
        const ST *K_ = Ks + buf * Gm::RE, *V_ = Vt + buf * (BF16 ? Gm::RE : Gm::TE);
        const float *bs = bias_s + buf * kTile;
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            // bf16: the running max enters as the accumulator's start (S^T - m out of the MFMA; this also
            // shortened the live ranges enough for three workgroups per CU); m = -inf before the first
            // sub-tile, whose start is 0
            const bool first = m == -INFINITY;  // wave-uniform (every lane starts there)
            f32x16 sacc;
#pragma unroll
            for (int v = 0; v < 16; ++v) sacc[v] = (BF16 && !first) ? -m : 0.f;
            mma_rows<BF16, D>(sacc, K_, sub * 32 + lr, lh, qf);  // S^T: rows = keys, col = this lane's query
            float s[16], bv[16], mx = -INFINITY;
            if constexpr (TB) crow_load16(bs + sub * 32, lh, bv);
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                s[v] = BF16 ? sacc[v] : sacc[v] * sl2;
                if constexpr (TB) s[v] += bv[v];
                mx = fmaxf(mx, s[v]);
            }
            mx = half_max(mx);
            if constexpr (BF16) {  // s holds S - m (first: S)
                if (first) {
                    m = mx;
#pragma unroll
                    for (int v = 0; v < 16; ++v) s[v] -= mx;
                } else if (__any(mx > kDefer)) {
                    const float up = fmaxf(mx, 0.f), corr = fast_exp2(-up);
                    l *= corr;
#pragma unroll
                    for (int t = 0; t < Gm::NT; ++t)
#pragma unroll
                        for (int v = 0; v < 16; ++v) acc[t][v] *= corr;
#pragma unroll
                    for (int v = 0; v < 16; ++v) s[v] -= up;
                    m += up;
                }
            } else {
                if (__any(mx > m + kDefer)) {  // m = -inf before the first sub-tile: always taken there
                    const float m_new = fmaxf(m, mx);
                    const float corr = fast_exp2(m - m_new);
                    l *= corr;
#pragma unroll
                    for (int t = 0; t < Gm::NT; ++t)
#pragma unroll
                        for (int v = 0; v < 16; ++v) acc[t][v] *= corr;
                    m = m_new;
                }
#pragma unroll
                for (int v = 0; v < 16; ++v) s[v] -= m;
            }
            float rs = 0.f;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                s[v] = fast_exp2(s[v]);
                rs += s[v];
            }
            l += half_sum(rs);
            if (drop) {  // dropout on the probabilities (the normalizer l keeps the undropped sum)
#pragma unroll
                for (int v = 0; v < 16; ++v)
                    s[v] = mtts::dropout_keep(s0, s1, prow, (uint32_t)(k0 + sub * 32 + crow(v, lh)), p.dropout_p)
                               ? s[v] * inv_keep
                               : 0.f;
            }
#pragma unroll
            for (int t = 0; t < Gm::NT; ++t) mma_perm<BF16, D>(acc[t], V_, t * 32 + lr, sub, lh, s);  // O^T += V^T P^T
        }
    };
    auto compute = [&](int buf, int k0) __attribute__((always_inline)) {  // tiles inside the valid keys skip the bias (wave-uniform)
        if (flag_s[buf])
            body(buf, k0, std::true_type{});
        else
            body(buf, k0, std::false_type{});
    };
    tile_loop<NB>((T + kTile - 1) / kTile, load, store, compute);

    if (q_ok) {
        const float inv = 1.f / l;
        TI *orow = Op + ((size_t)b * T + q) * p.ldo + h * dh;
#pragma unroll
        for (int t = 0; t < Gm::NT; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                if (t * 32 + 8 * g + 4 * lh < dh)
                    st4f(orow + t * 32 + 8 * g + 4 * lh,
                         make_float4(acc[t][4 * g] * inv, acc[t][4 * g + 1] * inv, acc[t][4 * g + 2] * inv,
                                     acc[t][4 * g + 3] * inv));
        if (lh == 0) p.lse[((size_t)b * p.H + h) * T + q] = m + log2f(l);
    }
}

// ------------------------------------------------------------------------------------------------
// dsum = rowsum(dO * O) over this lane's half of the head dims, then the two halves -- one function for
// the dQ pass and the Drow pre-pass, so both form the same value
template <int D, typename TI>
__device__ __forceinline__ float row_dot(const TI *orow, const TI *grow, int lh, int dh, bool ok) {
    float dsum = 0.f;
    if (ok) {
        orow += (D / 2) * lh;
        grow += (D / 2) * lh;
#pragma unroll
        for (int i = 0; i < D / 2; i += 4) {
            if ((D / 2) * lh + i >= dh) break;
            const float4 a = ld4f(orow + i);
            const float4 c = ld4f(grow + i);
            dsum += a.x * c.x + a.y * c.y + a.z * c.z + a.w * c.w;
        }
    }
    return half_sum(dsum);
}

// backward, dQ: grid (ceil(T/128), H, B); lane = query.  Writes Drow = rowsum(dO * O) for dKV unless the
// pre-pass did (Drow null).  bx: this workgroup's query block.
template <bool BF16, int D, typename TI, bool DROP>
__device__ __forceinline__ void bwd_dq_body(const mtts_attn_args &p, const mtts_attn_grads &g, float *Drow, int bx) {
    const TI *Qp = reinterpret_cast<const TI *>(p.q), *Kp = reinterpret_cast<const TI *>(p.k),
             *Vp = reinterpret_cast<const TI *>(p.v), *Op = reinterpret_cast<const TI *>(p.o),
             *Gp = reinterpret_cast<const TI *>(g.dout);
    TI *DQp = reinterpret_cast<TI *>(g.dq);
    using Gm = G<BF16, D>;
    using ST = typename Gm::T;
    constexpr int NB = nbuf(dq_stage<BF16, D>());
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char *sp = smem;
    ST *Ks = carve<ST>(sp, NB * Gm::RE);
    ST *Vs = carve<ST>(sp, NB * Gm::RE);
    ST *Kt = BF16 ? Ks : carve<ST>(sp, NB * Gm::TE);  // bf16: K^T is read from the K image
    float *bias_s = carve<float>(sp, NB * kTile);
    int *flag_s = carve<int>(sp, NB);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int3 bk_ = xcd_blk3();
    const int b = bk_.z, h = bk_.y, T = p.T, dh = p.D;  // dh <= D: columns past dh are zero
    const int q = bx * kRowsPerBlock + wave * 32 + lr;
    const bool q_ok = q < T;
    const size_t qrow = (size_t)b * T + (q_ok ? q : 0);
    const TI *Kb = Kp + h * dh, *Vb = Vp + h * dh;

    const float sl2 = p.scale * kLog2e, c0 = key_bias_c0(p, b);
    RowFrag<BF16, D> qf, gf;
    qf.load(Qp + h * dh + qrow * p.ldq, q_ok, lh, dh, BF16 ? sl2 : 1.f);  // as the forward's
    gf.load(Gp + h * dh + qrow * g.lddo, q_ok, lh, dh);
    // Drow[q] = sum_d dO[q,d] * O[q,d]: each half-wave lane sums D/2 dims
    const float dsum = row_dot<D>(Op + qrow * p.ldo + h * dh, Gp + qrow * g.lddo + h * dh, lh, dh, q_ok);
    const size_t srow = ((size_t)b * p.H + h) * T + (q_ok ? q : 0);
    const float lse2 = q_ok ? p.lse[srow] : 0.f;
    if (Drow && q_ok && lh == 0) Drow[srow] = dsum;

    f32x16 acc[Gm::NT];
#pragma unroll
    for (int t = 0; t < Gm::NT; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[t][v] = 0.f;

    TileLoader<BF16, D, TI> lk, lv;
    float bias_r = 0.f;
    auto load = [&](int k0) __attribute__((always_inline)) {
        lk.load(Kb, p.ldq, b, T, k0, tid, dh);
        lv.load(Vb, p.ldq, b, T, k0, tid, dh);
        bias_r = stage_bias(p, b, k0 + (tid & (kTile - 1)), c0);
    };
    auto store = [&](int buf) __attribute__((always_inline)) {
        lk.store(Ks + buf * Gm::RE, BF16 ? nullptr : Kt + buf * Gm::TE, tid, dh);
        lv.store(Vs + buf * Gm::RE, nullptr, tid, dh);
        store_bias(bias_s, flag_s, buf, bias_r, tid);
    };
    const bool drop = DROP && p.dropout_p > 0.f;  // DROP = false: no dropout code
    uint32_t s0 = 0, s1 = 0;
    if (drop) {
        s0 = p.seed[0];
        s1 = p.seed[1];
    }
    const float inv_keep = mtts::dropout_scale(p.dropout_p);
    const uint32_t prow = (uint32_t)srow;
    // bf16 without dropout: the row constants start the accumulators (S^T - lse, dP^T - D), so the
    // chains end ready for exp2 and the product
    const bool fold = BF16 && !drop;
    auto body = [&](int buf, int k0, auto has_bias) __attribute__((always_inline)) {
        constexpr bool TB = decltype(has_bias)::value;
        const ST *K_ = Ks + buf * Gm::RE, *V_ = Vs + buf * Gm::RE, *KT_ = BF16 ? K_ : Kt + buf * Gm::TE;
        const float *bs = bias_s + buf * kTile;
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            f32x16 sacc, pacc;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                sacc[v] = BF16 ? -lse2 : 0.f;
                pacc[v] = fold ? -dsum : 0.f;
            }
            mma_rows<BF16, D>(sacc, K_, sub * 32 + lr, lh, qf);  // S^T
            mma_rows<BF16, D>(pacc, V_, sub * 32 + lr, lh, gf);  // dP^T = V dO^T
            float ds[16], bv[16];
            if constexpr (TB) crow_load16(bs + sub * 32, lh, bv);
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                float x = BF16 ? sacc[v] : sacc[v] * sl2 - lse2;
                if constexpr (TB) x += bv[v];
                const float pr = fast_exp2(x);
                if (fold) {
                    ds[v] = pr * pacc[v];
                } else {
                    float dp = pacc[v];  // dL/d(dropped P) -> dL/dP through the regenerated mask
                    if (drop)
                        dp = mtts::dropout_keep(s0, s1, prow, (uint32_t)(k0 + sub * 32 + crow(v, lh)), p.dropout_p)
                                 ? dp * inv_keep
                                 : 0.f;
                    ds[v] = pr * (dp - dsum);
                }
            }
#pragma unroll
            for (int t = 0; t < Gm::NT; ++t) mma_perm<BF16, D>(acc[t], KT_, t * 32 + lr, sub, lh, ds);  // dQ^T += K^T dS^T
        }
    };
    auto compute = [&](int buf, int k0) __attribute__((always_inline)) {
        if (flag_s[buf])
            body(buf, k0, std::true_type{});
        else
            body(buf, k0, std::false_type{});
    };
    tile_loop<NB>((T + kTile - 1) / kTile, load, store, compute);

    if (q_ok) {
        TI *drow = DQp + ((size_t)b * T + q) * g.ldd + h * dh;
        const float sc = p.scale;
#pragma unroll
        for (int t = 0; t < Gm::NT; ++t)
#pragma unroll
            for (int gi = 0; gi < 4; ++gi)
                if (t * 32 + 8 * gi + 4 * lh < dh)
                    st4f(drow + t * 32 + 8 * gi + 4 * lh,
                         make_float4(acc[t][4 * gi] * sc, acc[t][4 * gi + 1] * sc, acc[t][4 * gi + 2] * sc,
                                     acc[t][4 * gi + 3] * sc));
    }
}

// ------------------------------------------------------------------------------------------------
// backward, dK/dV: grid (ceil(T/128), H, B); lane = key.  C layout: rows = queries, col = key.
template <bool BF16, int D, typename TI, bool DROP>
__device__ __forceinline__ void bwd_dkv_body(const mtts_attn_args &p, const mtts_attn_grads &g, const float *Drow, int bx) {
    const TI *Qp = reinterpret_cast<const TI *>(p.q), *Kp = reinterpret_cast<const TI *>(p.k),
             *Vp = reinterpret_cast<const TI *>(p.v), *Gp = reinterpret_cast<const TI *>(g.dout);
    TI *DKp = reinterpret_cast<TI *>(g.dk), *DVp = reinterpret_cast<TI *>(g.dv);
    using Gm = G<BF16, D>;
    using ST = typename Gm::T;
    constexpr int NB = nbuf(dkv_stage<BF16, D>());
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char *sp = smem;
    ST *Qs = carve<ST>(sp, NB * Gm::RE);
    ST *Gs = carve<ST>(sp, NB * Gm::RE);  // dO rows
    ST *Qt = BF16 ? Qs : carve<ST>(sp, NB * Gm::TE);  // bf16: transposed reads of the row images
    ST *Gt = BF16 ? Gs : carve<ST>(sp, NB * Gm::TE);  // dO transposed
    float *lse_s = carve<float>(sp, NB * kTile);  // +inf past T
    float *d_s = carve<float>(sp, NB * kTile);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int3 bk_ = xcd_blk3();
    const int b = bk_.z, h = bk_.y, T = p.T, dh = p.D;  // dh <= D: columns past dh are zero
    const int key = bx * kRowsPerBlock + wave * 32 + lr;
    const bool k_ok = key < T;
    const size_t krow = (size_t)b * T + (k_ok ? key : 0);

    const float sl2 = p.scale * kLog2e, c0 = key_bias_c0(p, b);
    RowFrag<BF16, D> kf, vf;
    kf.load(Kp + h * dh + krow * p.ldq, k_ok, lh, dh, BF16 ? sl2 : 1.f);  // bf16: S in the log2 domain
    vf.load(Vp + h * dh + krow * p.ldq, k_ok, lh, dh);
    const float bias2 = (k_ok && p.key_bias) ? (p.key_bias[krow] - c0) * kLog2e : 0.f;
    const TI *Qb = Qp + h * dh, *Gb = Gp + h * dh;
    const size_t sbase = ((size_t)b * p.H + h) * T;

    f32x16 dk[Gm::NT], dv[Gm::NT];
#pragma unroll
    for (int t = 0; t < Gm::NT; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) dk[t][v] = dv[t][v] = 0.f;

    TileLoader<BF16, D, TI> lq, lg;
    float lse_r = 0.f, d_r = 0.f;
    auto load = [&](int q0) __attribute__((always_inline)) {
        lq.load(Qb, p.ldq, b, T, q0, tid, dh);
        lg.load(Gb, g.lddo, b, T, q0, tid, dh);
        {
            const int qq = q0 + (tid & (kTile - 1));
            const float l_raw = p.lse[sbase + min(qq, T - 1)], d_raw = Drow[sbase + min(qq, T - 1)];
            lse_r = qq < T ? l_raw : INFINITY;
            d_r = qq < T ? d_raw : 0.f;
        }
    };
    auto store = [&](int buf) __attribute__((always_inline)) {
        lq.store(Qs + buf * Gm::RE, BF16 ? nullptr : Qt + buf * Gm::TE, tid, dh);
        lg.store(Gs + buf * Gm::RE, BF16 ? nullptr : Gt + buf * Gm::TE, tid, dh);
        if (tid < kTile) {
            lse_s[buf * kTile + tid] = lse_r;
            d_s[buf * kTile + tid] = d_r;
        }
    };
    const bool drop = DROP && p.dropout_p > 0.f;  // DROP = false: no dropout code
    uint32_t s0 = 0, s1 = 0;
    if (drop) {
        s0 = p.seed[0];
        s1 = p.seed[1];
    }
    const float inv_keep = mtts::dropout_scale(p.dropout_p);
    const bool fold = BF16 && !drop;  // row constants start the accumulators (as in the dQ kernel)
    auto compute = [&](int buf, int q0) __attribute__((always_inline)) {
        const ST *Q_ = Qs + buf * Gm::RE, *G_ = Gs + buf * Gm::RE;
        const ST *QT_ = BF16 ? Q_ : Qt + buf * Gm::TE, *GT_ = BF16 ? G_ : Gt + buf * Gm::TE;
        const float *ls = lse_s + buf * kTile, *dd = d_s + buf * kTile;
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            f32x16 sacc, pacc;
            float lv[16], dv16[16];
            crow_load16(ls + sub * 32, lh, lv);
            crow_load16(dd + sub * 32, lh, dv16);
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                sacc[v] = BF16 ? bias2 - lv[v] : 0.f;
                pacc[v] = fold ? -dv16[v] : 0.f;
            }
            mma_rows<BF16, D>(sacc, Q_, sub * 32 + lr, lh, kf);  // S = Q K^T (rows q, col = this key)
            mma_rows<BF16, D>(pacc, G_, sub * 32 + lr, lh, vf);  // dP = dO V^T
            float pr[16], ds[16];
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int qi = sub * 32 + crow(v, lh);
                const float pv = fast_exp2(BF16 ? sacc[v] : sacc[v] * sl2 + bias2 - lv[v]);
                pr[v] = pv;
                if (fold) {
                    ds[v] = pv * pacc[v];
                } else {
                    float dp = pacc[v];
                    if (drop) {  // P feeds dV through the forward's dropout mask
                        const bool keep =
                            mtts::dropout_keep(s0, s1, (uint32_t)(sbase + q0 + qi), (uint32_t)key, p.dropout_p);
                        pr[v] = keep ? pv * inv_keep : 0.f;
                        dp = keep ? dp * inv_keep : 0.f;
                    }
                    ds[v] = pv * (dp - dv16[v]);
                }
            }
#pragma unroll
            for (int t = 0; t < Gm::NT; ++t) {
                mma_perm<BF16, D>(dv[t], GT_, t * 32 + lr, sub, lh, pr);  // dV^T += dO^T P
                mma_perm<BF16, D>(dk[t], QT_, t * 32 + lr, sub, lh, ds);  // dK^T += Q^T dS
            }
        }
    };
    tile_loop<NB>((T + kTile - 1) / kTile, load, store, compute);

    if (k_ok) {
        TI *dkr = DKp + krow * g.ldd + h * dh;
        TI *dvr = DVp + krow * g.ldd + h * dh;
        const float sc = p.scale;
#pragma unroll
        for (int t = 0; t < Gm::NT; ++t)
#pragma unroll
            for (int gi = 0; gi < 4; ++gi) {
                const int c = t * 32 + 8 * gi + 4 * lh;
                if (c >= dh) continue;
                st4f(dkr + c, make_float4(dk[t][4 * gi] * sc, dk[t][4 * gi + 1] * sc, dk[t][4 * gi + 2] * sc,
                                          dk[t][4 * gi + 3] * sc));
                st4f(dvr + c, make_float4(dv[t][4 * gi], dv[t][4 * gi + 1], dv[t][4 * gi + 2], dv[t][4 * gi + 3]));
            }
    }
}

template <bool BF16, int D, typename TI = float, bool DROP = true>
__global__ __launch_bounds__(kThreads, D <= 64 ? 2 : 1) void attn_bwd_dq_kernel(mtts_attn_args p, mtts_attn_grads g, float *Drow) {
    bwd_dq_body<BF16, D, TI, DROP>(p, g, Drow, xcd_blk3().x);
}
template <bool BF16, int D, typename TI = float, bool DROP = true>
__global__ __launch_bounds__(kThreads, (BF16 && D <= 64) ? 2 : 1) void attn_bwd_dkv_kernel(mtts_attn_args p, mtts_attn_grads g,
                                                                                        const float *Drow) {
    bwd_dkv_body<BF16, D, TI, DROP>(p, g, Drow, xcd_blk3().x);
}

// Drow pre-pass: rowsum(dO * O) per (query, head), grid (ceil(T/128), H, B), the dQ pass's lane mapping
// and summation (row_dot) -- so the merged backward below needs no ordering between its two halves
template <int D, typename TI>
__global__ __launch_bounds__(kThreads) void attn_drow_kernel(mtts_attn_args p, mtts_attn_grads g, float *Drow) {
    const TI *Op = reinterpret_cast<const TI *>(p.o), *Gp = reinterpret_cast<const TI *>(g.dout);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int3 bk_ = xcd_blk3();
    const int b = bk_.z, h = bk_.y, T = p.T, dh = p.D;
    const int q = bk_.x * kRowsPerBlock + wave * 32 + lr;
    const bool q_ok = q < T;
    const size_t qrow = (size_t)b * T + (q_ok ? q : 0);
    const float dsum = row_dot<D>(Op + qrow * p.ldo + h * dh, Gp + qrow * g.lddo + h * dh, lh, dh, q_ok);
    if (q_ok && lh == 0) Drow[((size_t)b * p.H + h) * T + q] = dsum;
}

// Merged backward: grid (2 * nq, H, B) -- the first nq workgroups run the dQ pass, the rest the dK/dV pass
// (Drow from the pre-pass).  One launch of twice the workgroups: at T = 600 the 640 + 640 workgroups fill
// ~2.5 rounds of the 512 slots instead of 2 + 2.
template <bool BF16, int D, typename TI = float, bool DROP = true>
__global__ __launch_bounds__(kThreads, (BF16 && D <= 64) ? 2 : 1) void attn_bwd_merged_kernel(mtts_attn_args p, mtts_attn_grads g,
                                                                                           float *Drow, int nq) {
    const int bx = xcd_blk3().x;
    if (bx < nq) bwd_dq_body<BF16, D, TI, DROP>(p, g, nullptr, bx);
    else bwd_dkv_body<BF16, D, TI, DROP>(p, g, Drow, bx - nq);
}

// ------------------------------------------------------------------------------------------------
// Short sequences (T <= 128: the text encoder, T ~ 120 x 2 heads of 96).  The kernels above give a
// (b, h) pair one block of 128 rows, so the encoder's 64 pairs fill a quarter of the chip and each block
// walks its two 64-row tiles in series.  Here a block owns 32 rows and its four waves split the OTHER
// axis -- wave w takes the 32 keys (fwd, dQ) or queries (dKV) of sub-tile w -- with both tiles staged
// at once; the waves' partial results are merged through LDS in wave order (deterministic).  4x the
// blocks, a quarter of the serial chain per block.  fp32 reads its transposed operands from the row
// tiles (no transposed copies), which keeps two tiles of two operands inside the LDS.
constexpr int kShortT = 2 * kTile;
constexpr int kShortRows = 32;

template <bool BF16, int D>
struct Short {
    using Gm = G<BF16, D>;
    static constexpr size_t tile = ((size_t)Gm::RE * sizeof(typename Gm::T) + 15) / 16 * 16;
    static constexpr size_t stage = 4 * tile + 2 * (2 * kTile * sizeof(float)) + 16;  // 2 tiles x 2 operands + 2 row arrays
    static constexpr size_t acc_set = (size_t)kWaves * Gm::NT * 16 * 64 * sizeof(float);  // one wave-partial accumulator set
    static constexpr size_t xoff(int nacc) { return stage > nacc * acc_set ? stage : nacc * acc_set; }
    static constexpr size_t lds(int nacc) { return xoff(nacc) + 2 * kWaves * 32 * sizeof(float) + 64; }
};

// mma_perm on a ROW tile: bf16 images are read transposed by the same call; fp32 indexes the row tile
// by (key, d) instead of a transposed copy's (d, key)
template <bool BF16, int D>
__device__ __forceinline__ void mma_perm_r(f32x16 &acc, const typename G<BF16, D>::T *tile, int d, int sub, int lh,
                                           const float (&s)[16]) {
    if constexpr (BF16) {
        mma_perm<BF16, D>(acc, tile, d, sub, lh, s);
    } else {
        constexpr int LD = G<BF16, D>::LDR;
#pragma unroll
        for (int v = 0; v < 16; ++v)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(tile[(sub * 32 + crow(v, lh)) * LD + d], s[v], acc, 0, 0, 0);
    }
}

// both 64-row tiles of two operands (rows 0..127 of one head) into LDS; rows past T hold finite data
// that every kernel weights by zero (as TileLoader)
template <bool BF16, int D, typename TI>
__device__ __forceinline__ void stage_pair(const TI *A, const TI *Bm, int lda, int ldb, int b, int T, int tid, int dh,
                                           typename G<BF16, D>::T *As, typename G<BF16, D>::T *Bs) {
    using Gm = G<BF16, D>;
    TileLoader<BF16, D, TI> la0, lb0, la1, lb1;
    la0.load(A, lda, b, T, 0, tid, dh);
    lb0.load(Bm, ldb, b, T, 0, tid, dh);
    const bool two = T > kTile;
    if (two) {
        la1.load(A, lda, b, T, kTile, tid, dh);
        lb1.load(Bm, ldb, b, T, kTile, tid, dh);
    }
    la0.store(As, nullptr, tid, dh);
    lb0.store(Bs, nullptr, tid, dh);
    if (two) {
        la1.store(As + Gm::RE, nullptr, tid, dh);
        lb1.store(Bs + Gm::RE, nullptr, tid, dh);
    }
}

// The wave-partial accumulators of this wave into the merge area: [wave][t][v][lane] (lane-contiguous)
template <int NT>
__device__ __forceinline__ void put_partial(float *area, const f32x16 (&acc)[NT], int wave, int lane) {
    float *mine = area + (size_t)wave * NT * 16 * 64;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) mine[(t * 16 + v) * 64 + lane] = acc[t][v];
}
// sum over waves (fixed order, weights wgt[w]) of the C-layout values 4g..4g+3 of tile t
template <int NT>
__device__ __forceinline__ float4 sum_partials(const float *area, int t, int g, int lane, const float (&wgt)[kWaves]) {
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        const float *pw = area + (size_t)w * NT * 16 * 64 + (t * 16 + 4 * g) * 64 + lane;
        o.x += wgt[w] * pw[0];
        o.y += wgt[w] * pw[64];
        o.z += wgt[w] * pw[128];
        o.w += wgt[w] * pw[192];
    }
    return o;
}

// forward: grid (ceil(T/32), H, B); lane = query, wave = key sub-tile
template <bool BF16, int D, typename TI = float>
__global__ __launch_bounds__(kThreads) void attn_fwd_short_kernel(mtts_attn_args p) {
    const TI *Qp = reinterpret_cast<const TI *>(p.q), *Kp = reinterpret_cast<const TI *>(p.k),
             *Vp = reinterpret_cast<const TI *>(p.v);
    TI *Op = reinterpret_cast<TI *>(p.o);
    using Gm = G<BF16, D>;
    using ST = typename Gm::T;
    using S = Short<BF16, D>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char *sp = smem;
    ST *Ks = carve<ST>(sp, 2 * Gm::RE);
    ST *Vs = carve<ST>(sp, 2 * Gm::RE);
    float *bias_s = carve<float>(sp, 2 * kTile);
    int *flag_s = carve<int>(sp, 2);
    float *area = reinterpret_cast<float *>(smem);  // merge area: aliases the stage after the compute
    float *ms = reinterpret_cast<float *>(smem + S::xoff(1)), *ls = ms + kWaves * 32;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int3 bk_ = xcd_blk3();
    const int b = bk_.z, h = bk_.y, T = p.T, dh = p.D;
    const int q = bk_.x * kShortRows + lr;
    const bool q_ok = q < T;
    const int buf = wave >> 1, sub = wave & 1;
    const float c0 = key_bias_c0(p, b), sl2 = p.scale * kLog2e;

    RowFrag<BF16, D> qf;
    qf.load(Qp + h * dh + ((size_t)b * T + (q_ok ? q : 0)) * p.ldq, q_ok, lh, dh, BF16 ? sl2 : 1.f);
    const float br0 = stage_bias(p, b, tid & (kTile - 1), c0), br1 = stage_bias(p, b, kTile + (tid & (kTile - 1)), c0);
    stage_pair<BF16, D>(Kp + h * dh, Vp + h * dh, p.ldq, p.ldq, b, T, tid, dh, Ks, Vs);
    store_bias(bias_s, flag_s, 0, br0, tid);
    store_bias(bias_s, flag_s, 1, br1, tid);
    mtts::lds_barrier();

    f32x16 acc[Gm::NT];
#pragma unroll
    for (int t = 0; t < Gm::NT; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[t][v] = 0.f;
    float m = -INFINITY, l = 0.f;
    if (wave * 32 < T) {  // wave-uniform: the sub-tile holds at least one key (so m is finite)
        const ST *K_ = Ks + buf * Gm::RE, *V_ = Vs + buf * Gm::RE;
        f32x16 sacc;
#pragma unroll
        for (int v = 0; v < 16; ++v) sacc[v] = 0.f;
        mma_rows<BF16, D>(sacc, K_, sub * 32 + lr, lh, qf);
        float s[16], bv[16], mx = -INFINITY;
        const bool tb = flag_s[buf];
        if (tb) crow_load16(bias_s + buf * kTile + sub * 32, lh, bv);
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            s[v] = BF16 ? sacc[v] : sacc[v] * sl2;
            if (tb) s[v] += bv[v];
            mx = fmaxf(mx, s[v]);
        }
        m = half_max(mx);
        float rs = 0.f;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            s[v] = fast_exp2(s[v] - m);
            rs += s[v];
        }
        l = half_sum(rs);
        if (p.dropout_p > 0.f) {
            const uint32_t s0 = p.seed[0], s1 = p.seed[1];
            const uint32_t prow = (uint32_t)(((size_t)b * p.H + h) * T + q);
            const float inv_keep = mtts::dropout_scale(p.dropout_p);
#pragma unroll
            for (int v = 0; v < 16; ++v)
                s[v] = mtts::dropout_keep(s0, s1, prow, (uint32_t)(wave * 32 + crow(v, lh)), p.dropout_p)
                           ? s[v] * inv_keep
                           : 0.f;
        }
#pragma unroll
        for (int t = 0; t < Gm::NT; ++t) mma_perm_r<BF16, D>(acc[t], V_, t * 32 + lr, sub, lh, s);
    }
    mtts::lds_barrier();  // the staged tiles are dead: the merge area may overwrite them
    if (lh == 0) {
        ms[wave * 32 + lr] = m;
        ls[wave * 32 + lr] = l;
    }
    put_partial<Gm::NT>(area, acc, wave, lane);
    mtts::lds_barrier();
    float M = -INFINITY, L = 0.f, wgt[kWaves];
#pragma unroll
    for (int w = 0; w < kWaves; ++w) M = fmaxf(M, ms[w * 32 + lr]);
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        const float mw = ms[w * 32 + lr];
        wgt[w] = mw == -INFINITY ? 0.f : fast_exp2(mw - M);
        L += wgt[w] * ls[w * 32 + lr];
    }
    if (q_ok) {
        const float inv = 1.f / L;
        TI *orow = Op + ((size_t)b * T + q) * p.ldo + h * dh;
#pragma unroll
        for (int t = 0; t < Gm::NT; ++t) {
            const int c = t * 32 + 8 * wave + 4 * lh;  // wave w writes the C-layout group g = w
            if (c >= dh) continue;
            const float4 o = sum_partials<Gm::NT>(area, t, wave, lane, wgt);
            st4f(orow + c, make_float4(o.x * inv, o.y * inv, o.z * inv, o.w * inv));
        }
        if (wave == 0 && lh == 0) p.lse[((size_t)b * p.H + h) * T + q] = M + log2f(L);
    }
}

// backward dQ: grid (ceil(T/32), H, B); lane = query, wave = key sub-tile.  Writes Drow as well.
template <bool BF16, int D, typename TI = float>
__global__ __launch_bounds__(kThreads) void attn_bwd_dq_short_kernel(mtts_attn_args p, mtts_attn_grads g, float *Drow) {
    const TI *Qp = reinterpret_cast<const TI *>(p.q), *Kp = reinterpret_cast<const TI *>(p.k),
             *Vp = reinterpret_cast<const TI *>(p.v), *Op = reinterpret_cast<const TI *>(p.o),
             *Gp = reinterpret_cast<const TI *>(g.dout);
    TI *DQp = reinterpret_cast<TI *>(g.dq);
    using Gm = G<BF16, D>;
    using ST = typename Gm::T;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char *sp = smem;
    ST *Ks = carve<ST>(sp, 2 * Gm::RE);
    ST *Vs = carve<ST>(sp, 2 * Gm::RE);
    float *bias_s = carve<float>(sp, 2 * kTile);
    int *flag_s = carve<int>(sp, 2);
    float *area = reinterpret_cast<float *>(smem);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int3 bk_ = xcd_blk3();
    const int b = bk_.z, h = bk_.y, T = p.T, dh = p.D;
    const int q = bk_.x * kShortRows + lr;
    const bool q_ok = q < T;
    const size_t qrow = (size_t)b * T + (q_ok ? q : 0);
    const int buf = wave >> 1, sub = wave & 1;
    const float sl2 = p.scale * kLog2e, c0 = key_bias_c0(p, b);

    RowFrag<BF16, D> qf, gf;
    qf.load(Qp + h * dh + qrow * p.ldq, q_ok, lh, dh, BF16 ? sl2 : 1.f);
    gf.load(Gp + h * dh + qrow * g.lddo, q_ok, lh, dh);
    float dsum = 0.f;  // rowsum(dO * O), as the long dQ kernel (every wave: the same query per lane)
    if (q_ok) {
        const TI *orow = Op + qrow * p.ldo + h * dh + (D / 2) * lh;
        const TI *grow = Gp + qrow * g.lddo + h * dh + (D / 2) * lh;
#pragma unroll
        for (int i = 0; i < D / 2; i += 4) {
            if ((D / 2) * lh + i >= dh) break;
            const float4 a = ld4f(orow + i);
            const float4 c = ld4f(grow + i);
            dsum += a.x * c.x + a.y * c.y + a.z * c.z + a.w * c.w;
        }
    }
    dsum = half_sum(dsum);
    const size_t srow = ((size_t)b * p.H + h) * T + (q_ok ? q : 0);
    const float lse2 = q_ok ? p.lse[srow] : 0.f;
    if (q_ok && wave == 0 && lh == 0) Drow[srow] = dsum;

    const float br0 = stage_bias(p, b, tid & (kTile - 1), c0), br1 = stage_bias(p, b, kTile + (tid & (kTile - 1)), c0);
    stage_pair<BF16, D>(Kp + h * dh, Vp + h * dh, p.ldq, p.ldq, b, T, tid, dh, Ks, Vs);
    store_bias(bias_s, flag_s, 0, br0, tid);
    store_bias(bias_s, flag_s, 1, br1, tid);
    mtts::lds_barrier();

    f32x16 acc[Gm::NT];
#pragma unroll
    for (int t = 0; t < Gm::NT; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[t][v] = 0.f;
    if (wave * 32 < T) {
        const bool drop = p.dropout_p > 0.f, fold = BF16 && !drop;
        const ST *K_ = Ks + buf * Gm::RE, *V_ = Vs + buf * Gm::RE;
        f32x16 sacc, pacc;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            sacc[v] = BF16 ? -lse2 : 0.f;
            pacc[v] = fold ? -dsum : 0.f;
        }
        mma_rows<BF16, D>(sacc, K_, sub * 32 + lr, lh, qf);  // S^T
        mma_rows<BF16, D>(pacc, V_, sub * 32 + lr, lh, gf);  // dP^T
        float ds[16], bv[16];
        const bool tb = flag_s[buf];
        if (tb) crow_load16(bias_s + buf * kTile + sub * 32, lh, bv);
        const uint32_t s0 = drop ? p.seed[0] : 0u, s1 = drop ? p.seed[1] : 0u;
        const float inv_keep = mtts::dropout_scale(p.dropout_p);
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            float x = BF16 ? sacc[v] : sacc[v] * sl2 - lse2;
            if (tb) x += bv[v];
            const float pr = fast_exp2(x);
            if (fold) {
                ds[v] = pr * pacc[v];
            } else {
                float dp = pacc[v];
                if (drop)
                    dp = mtts::dropout_keep(s0, s1, (uint32_t)srow, (uint32_t)(wave * 32 + crow(v, lh)), p.dropout_p)
                             ? dp * inv_keep
                             : 0.f;
                ds[v] = pr * (dp - dsum);
            }
        }
#pragma unroll
        for (int t = 0; t < Gm::NT; ++t) mma_perm_r<BF16, D>(acc[t], K_, t * 32 + lr, sub, lh, ds);  // dQ^T += K^T dS^T
    }
    mtts::lds_barrier();
    put_partial<Gm::NT>(area, acc, wave, lane);
    mtts::lds_barrier();
    if (q_ok) {
        const float one[kWaves] = {1.f, 1.f, 1.f, 1.f};
        TI *drow = DQp + ((size_t)b * T + q) * g.ldd + h * dh;
        const float sc = p.scale;
#pragma unroll
        for (int t = 0; t < Gm::NT; ++t) {
            const int c = t * 32 + 8 * wave + 4 * lh;
            if (c >= dh) continue;
            const float4 o = sum_partials<Gm::NT>(area, t, wave, lane, one);
            st4f(drow + c, make_float4(o.x * sc, o.y * sc, o.z * sc, o.w * sc));
        }
    }
}

// backward dK/dV: grid (ceil(T/32), H, B); lane = key, wave = query sub-tile
template <bool BF16, int D, typename TI = float>
__global__ __launch_bounds__(kThreads) void attn_bwd_dkv_short_kernel(mtts_attn_args p, mtts_attn_grads g,
                                                                      const float *Drow) {
    const TI *Qp = reinterpret_cast<const TI *>(p.q), *Kp = reinterpret_cast<const TI *>(p.k),
             *Vp = reinterpret_cast<const TI *>(p.v), *Gp = reinterpret_cast<const TI *>(g.dout);
    TI *DKp = reinterpret_cast<TI *>(g.dk), *DVp = reinterpret_cast<TI *>(g.dv);
    using Gm = G<BF16, D>;
    using ST = typename Gm::T;
    using S = Short<BF16, D>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char *sp = smem;
    ST *Qs = carve<ST>(sp, 2 * Gm::RE);
    ST *Gs = carve<ST>(sp, 2 * Gm::RE);
    float *lse_s = carve<float>(sp, 2 * kTile);  // +inf past T
    float *d_s = carve<float>(sp, 2 * kTile);
    float *area_k = reinterpret_cast<float *>(smem), *area_v = reinterpret_cast<float *>(smem + S::acc_set);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 31, lh = lane >> 5;
    const int3 bk_ = xcd_blk3();
    const int b = bk_.z, h = bk_.y, T = p.T, dh = p.D;
    const int key = bk_.x * kShortRows + lr;
    const bool k_ok = key < T;
    const size_t krow = (size_t)b * T + (k_ok ? key : 0);
    const int buf = wave >> 1, sub = wave & 1;
    const float sl2 = p.scale * kLog2e, c0 = key_bias_c0(p, b);

    RowFrag<BF16, D> kf, vf;
    kf.load(Kp + h * dh + krow * p.ldq, k_ok, lh, dh, BF16 ? sl2 : 1.f);
    vf.load(Vp + h * dh + krow * p.ldq, k_ok, lh, dh);
    const float bias2 = (k_ok && p.key_bias) ? (p.key_bias[krow] - c0) * kLog2e : 0.f;
    const size_t sbase = ((size_t)b * p.H + h) * T;
    float lse_r = 0.f, d_r = 0.f;
    if (tid < kShortT) {
        const float l_raw = p.lse[sbase + min(tid, T - 1)], d_raw = Drow[sbase + min(tid, T - 1)];
        lse_r = tid < T ? l_raw : INFINITY;
        d_r = tid < T ? d_raw : 0.f;
    }
    stage_pair<BF16, D>(Qp + h * dh, Gp + h * dh, p.ldq, g.lddo, b, T, tid, dh, Qs, Gs);
    if (tid < kShortT) {
        lse_s[tid] = lse_r;
        d_s[tid] = d_r;
    }
    mtts::lds_barrier();

    f32x16 dk[Gm::NT], dv[Gm::NT];
#pragma unroll
    for (int t = 0; t < Gm::NT; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) dk[t][v] = dv[t][v] = 0.f;
    if (wave * 32 < T) {
        const bool drop = p.dropout_p > 0.f, fold = BF16 && !drop;
        const ST *Q_ = Qs + buf * Gm::RE, *G_ = Gs + buf * Gm::RE;
        float lv[16], dv16[16];
        crow_load16(lse_s + wave * 32, lh, lv);
        crow_load16(d_s + wave * 32, lh, dv16);
        f32x16 sacc, pacc;
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            sacc[v] = BF16 ? bias2 - lv[v] : 0.f;
            pacc[v] = fold ? -dv16[v] : 0.f;
        }
        mma_rows<BF16, D>(sacc, Q_, sub * 32 + lr, lh, kf);  // S (rows q, col = this key)
        mma_rows<BF16, D>(pacc, G_, sub * 32 + lr, lh, vf);  // dP
        const uint32_t s0 = drop ? p.seed[0] : 0u, s1 = drop ? p.seed[1] : 0u;
        const float inv_keep = mtts::dropout_scale(p.dropout_p);
        float pr[16], ds[16];
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const float pv = fast_exp2(BF16 ? sacc[v] : sacc[v] * sl2 + bias2 - lv[v]);
            pr[v] = pv;
            if (fold) {
                ds[v] = pv * pacc[v];
            } else {
                float dp = pacc[v];
                if (drop) {
                    const bool keep = mtts::dropout_keep(s0, s1, (uint32_t)(sbase + wave * 32 + crow(v, lh)),
                                                         (uint32_t)key, p.dropout_p);
                    pr[v] = keep ? pv * inv_keep : 0.f;
                    dp = keep ? dp * inv_keep : 0.f;
                }
                ds[v] = pv * (dp - dv16[v]);
            }
        }
#pragma unroll
        for (int t = 0; t < Gm::NT; ++t) {
            mma_perm_r<BF16, D>(dv[t], G_, t * 32 + lr, sub, lh, pr);  // dV^T += dO^T P
            mma_perm_r<BF16, D>(dk[t], Q_, t * 32 + lr, sub, lh, ds);  // dK^T += Q^T dS
        }
    }
    mtts::lds_barrier();
    put_partial<Gm::NT>(area_k, dk, wave, lane);
    put_partial<Gm::NT>(area_v, dv, wave, lane);
    mtts::lds_barrier();
    if (k_ok) {
        const float one[kWaves] = {1.f, 1.f, 1.f, 1.f};
        TI *dkr = DKp + krow * g.ldd + h * dh;
        TI *dvr = DVp + krow * g.ldd + h * dh;
        const float sc = p.scale;
#pragma unroll
        for (int t = 0; t < Gm::NT; ++t) {
            const int c = t * 32 + 8 * wave + 4 * lh;
            if (c >= dh) continue;
            const float4 a = sum_partials<Gm::NT>(area_k, t, wave, lane, one);
            const float4 e = sum_partials<Gm::NT>(area_v, t, wave, lane, one);
            st4f(dkr + c, make_float4(a.x * sc, a.y * sc, a.z * sc, a.w * sc));
            st4f(dvr + c, e);
        }
    }
}

// the short path is the default for T <= 128; MTTS_ATTN_SHORT=0 sends every shape down the long one
bool use_short(int T) {
    if (T > kShortT) return false;
    const char *e = getenv("MTTS_ATTN_SHORT");
    return !(e && e[0] == '0');
}

constexpr size_t lds_bytes(size_t stage) { return nbuf(stage) * (stage + 64); }  // + carve alignment slack

template <typename K>
bool set_lds(K kernel, size_t bytes) {
    if (bytes <= 64 * 1024) return true;
    return hipFuncSetAttribute(reinterpret_cast<const void *>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes) == hipSuccess;
}

bool aligned16(const void *ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

int check_args(const mtts_attn_args *p, int precision) {
    MTTS_CHECK_ARG(p, "attention: null args");
    MTTS_CHECK_ARG(precision == MTTS_PREC_FP32 || precision == MTTS_PREC_BF16, "attention: bad precision");
    MTTS_CHECK_ARG(p->D >= 8 && p->D <= 96 && p->D % 8 == 0, "attention: head dim must be a multiple of 8 in [8, 96]");
    MTTS_CHECK_ARG(p->B >= 0 && p->T >= 0 && p->H >= 1, "attention: bad shape");
    MTTS_CHECK_ARG(p->q && p->k && p->v && p->o && p->lse, "attention: null tensor");
    MTTS_CHECK_ARG(p->ldq % 4 == 0 && p->ldo % 4 == 0 && p->ldq >= p->H * p->D && p->ldo >= p->H * p->D,
                   "attention: row strides must be multiples of 4 and cover H*D");
    MTTS_CHECK_ARG(aligned16(p->q) && aligned16(p->k) && aligned16(p->v) && aligned16(p->o),
                   "attention: q/k/v/o must be 16-byte aligned");
    MTTS_CHECK_ARG(p->scale > 0.f, "attention: scale must be positive");
    MTTS_CHECK_ARG(p->dropout_p >= 0.f && p->dropout_p < 1.f && (p->dropout_p == 0.f || p->seed),
                   "attention: dropout_p in [0, 1) with a seed");
    MTTS_CHECK_ARG(!(p->flags & ~MTTS_ATTN_F_IO_BF16), "attention: unknown flag");
    MTTS_CHECK_ARG(!(p->flags & MTTS_ATTN_F_IO_BF16) || precision == MTTS_PREC_BF16,
                   "attention: bf16 storage needs bf16 precision");
    return MTTS_OK;
}

template <bool BF16, int D, typename TI = float>
int fwd_launch(const mtts_attn_args &p, hipStream_t st) {
    if constexpr (BF16 && sizeof(TI) == 4) {
        if (p.flags & MTTS_ATTN_F_IO_BF16) return fwd_launch<true, D, uint16_t>(p, st);
    }
    if (use_short(p.T)) {
        constexpr size_t ls = Short<BF16, D>::lds(1);
        static_assert(ls <= kLdsMax, "attention short fwd LDS");
        if (!set_lds(attn_fwd_short_kernel<BF16, D, TI>, ls)) return mtts::fail(MTTS_ERR_HIP, "attention: LDS attribute");
        dim3 grid((p.T + kShortRows - 1) / kShortRows, p.H, p.B);
        hipLaunchKernelGGL((attn_fwd_short_kernel<BF16, D, TI>), grid, dim3(kThreads), ls, st, p);
        return mtts::check_launch("attn_fwd_short_kernel");
    }
    constexpr size_t lds = lds_bytes(fwd_stage<BF16, D>());
    static_assert(lds <= kLdsMax, "attention fwd LDS");
    const bool drop = p.dropout_p > 0.f;  // the dropout-free instance holds fewer registers
    if (!set_lds(attn_fwd_kernel<BF16, D, TI, true>, lds) || !set_lds(attn_fwd_kernel<BF16, D, TI, false>, lds))
        return mtts::fail(MTTS_ERR_HIP, "attention: LDS attribute");
    dim3 grid((p.T + kRowsPerBlock - 1) / kRowsPerBlock, p.H, p.B);
    if (drop) hipLaunchKernelGGL((attn_fwd_kernel<BF16, D, TI, true>), grid, dim3(kThreads), lds, st, p);
    else hipLaunchKernelGGL((attn_fwd_kernel<BF16, D, TI, false>), grid, dim3(kThreads), lds, st, p);
    return mtts::check_launch("attn_fwd_kernel");
}

// merged backward (default) or the two-launch dQ, dK/dV sequence (MTTS_ATTN_BWD_MERGED=0)
bool bwd_merged() {
    const char *e = getenv("MTTS_ATTN_BWD_MERGED");
    return !(e && e[0] == '0');
}

template <bool BF16, int D, typename TI = float>
int bwd_launch(const mtts_attn_args &p, const mtts_attn_grads &g, float *Drow, hipStream_t st) {
    if constexpr (BF16 && sizeof(TI) == 4) {
        if (p.flags & MTTS_ATTN_F_IO_BF16) return bwd_launch<true, D, uint16_t>(p, g, Drow, st);
    }
    if (use_short(p.T)) {
        constexpr size_t sq = Short<BF16, D>::lds(1), skv = Short<BF16, D>::lds(2);
        static_assert(sq <= kLdsMax && skv <= kLdsMax, "attention short bwd LDS");
        if (!set_lds(attn_bwd_dq_short_kernel<BF16, D, TI>, sq) || !set_lds(attn_bwd_dkv_short_kernel<BF16, D, TI>, skv))
            return mtts::fail(MTTS_ERR_HIP, "attention_bwd: LDS attribute");
        dim3 grid((p.T + kShortRows - 1) / kShortRows, p.H, p.B);
        hipLaunchKernelGGL((attn_bwd_dq_short_kernel<BF16, D, TI>), grid, dim3(kThreads), sq, st, p, g, Drow);
        if (int rc = mtts::check_launch("attn_bwd_dq_short_kernel")) return rc;
        hipLaunchKernelGGL((attn_bwd_dkv_short_kernel<BF16, D, TI>), grid, dim3(kThreads), skv, st, p, g,
                           (const float *)Drow);
        return mtts::check_launch("attn_bwd_dkv_short_kernel");
    }
    constexpr size_t lq = lds_bytes(dq_stage<BF16, D>()), lkv = lds_bytes(dkv_stage<BF16, D>());
    static_assert(lq <= kLdsMax && lkv <= kLdsMax, "attention bwd LDS");
    if (!set_lds(attn_bwd_dq_kernel<BF16, D, TI, true>, lq) || !set_lds(attn_bwd_dkv_kernel<BF16, D, TI, true>, lkv) ||
        !set_lds(attn_bwd_dq_kernel<BF16, D, TI, false>, lq) || !set_lds(attn_bwd_dkv_kernel<BF16, D, TI, false>, lkv))
        return mtts::fail(MTTS_ERR_HIP, "attention_bwd: LDS attribute");
    dim3 grid((p.T + kRowsPerBlock - 1) / kRowsPerBlock, p.H, p.B);
    const bool drop = p.dropout_p > 0.f;
    if (bwd_merged()) {  // Drow pre-pass, then the two passes as ONE launch
        constexpr size_t lm = lq > lkv ? lq : lkv;
        if (!set_lds(attn_bwd_merged_kernel<BF16, D, TI, true>, lm) || !set_lds(attn_bwd_merged_kernel<BF16, D, TI, false>, lm))
            return mtts::fail(MTTS_ERR_HIP, "attention_bwd: LDS attribute");
        hipLaunchKernelGGL((attn_drow_kernel<D, TI>), grid, dim3(kThreads), 0, st, p, g, Drow);
        if (int rc = mtts::check_launch("attn_drow_kernel")) return rc;
        const int nq = (int)grid.x;
        dim3 grid2(2 * grid.x, grid.y, grid.z);
        if (drop) hipLaunchKernelGGL((attn_bwd_merged_kernel<BF16, D, TI, true>), grid2, dim3(kThreads), lm, st, p, g, Drow, nq);
        else hipLaunchKernelGGL((attn_bwd_merged_kernel<BF16, D, TI, false>), grid2, dim3(kThreads), lm, st, p, g, Drow, nq);
        return mtts::check_launch("attn_bwd_merged_kernel");
    }
    if (drop) hipLaunchKernelGGL((attn_bwd_dq_kernel<BF16, D, TI, true>), grid, dim3(kThreads), lq, st, p, g, Drow);
    else hipLaunchKernelGGL((attn_bwd_dq_kernel<BF16, D, TI, false>), grid, dim3(kThreads), lq, st, p, g, Drow);
    if (int rc = mtts::check_launch("attn_bwd_dq_kernel")) return rc;
    if (drop)
        hipLaunchKernelGGL((attn_bwd_dkv_kernel<BF16, D, TI, true>), grid, dim3(kThreads), lkv, st, p, g, (const float *)Drow);
    else
        hipLaunchKernelGGL((attn_bwd_dkv_kernel<BF16, D, TI, false>), grid, dim3(kThreads), lkv, st, p, g, (const float *)Drow);
    return mtts::check_launch("attn_bwd_dkv_kernel");
}

template <bool BF16>
int fwd_dispatch(const mtts_attn_args &p, hipStream_t st) {
    return p.D <= 32 ? fwd_launch<BF16, 32>(p, st) : p.D <= 64 ? fwd_launch<BF16, 64>(p, st) : fwd_launch<BF16, 96>(p, st);
}
template <bool BF16>
int bwd_dispatch(const mtts_attn_args &p, const mtts_attn_grads &g, float *Drow, hipStream_t st) {
    return p.D <= 32   ? bwd_launch<BF16, 32>(p, g, Drow, st)
           : p.D <= 64 ? bwd_launch<BF16, 64>(p, g, Drow, st)
                       : bwd_launch<BF16, 96>(p, g, Drow, st);
}

// RoPE (text_encoder.py:99-143, rotate-half form) on the q and k column blocks of a fused [rows, 3C]
// projection, v copied: one thread per element.  Head dim D, rotated dims [0, R) of each head, half = R/2,
// cos/sin [T][half].  forward: y_d = x_d cos - x_{d+half} sin (d < half), x_d cos + x_{d-half} sin;
// inverse (the backward, R^T): the signs of the sin terms flip.
__global__ void rope_qk_kernel(const float *__restrict__ x, float *__restrict__ y, int rows, int T, int C, int D, int R,
                               const float *__restrict__ cs, const float *__restrict__ sn, float sgn) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int W = 3 * C;
    if (idx >= (int64_t)rows * W) return;
    const int r = (int)(idx / W), col = (int)(idx - (int64_t)r * W);
    const float *xr = x + (size_t)r * W;
    float v = xr[col];
    const int d = (col % C) % D;
    if (col < 2 * C && d < R) {
        const int half = R / 2, t = r % T;
        const int i = d < half ? d : d - half;
        const float c = cs[t * half + i], s = sn[t * half + i];
        v = d < half ? v * c - sgn * xr[col + half] * s : v * c + sgn * xr[col - half] * s;
    }
    y[(size_t)r * W + col] = v;
}

// Same rotation, four channels per thread (float4 loads / stores, 32-bit index math): a 4-column group
// never straddles a head, the rotated range or its halves when D, R / 2 and C are multiples of 4, and
// its partner group sits R / 2 columns away.  The scalar kernel (64-bit index division per element)
// ran at ~1.8 TB/s on the encoder's [3840, 576] q|k|v.
__global__ void rope_qk_vec4_kernel(const float4 *__restrict__ x, float4 *__restrict__ y, int rows, int T, int C,
                                    int D, int R, const float *__restrict__ cs, const float *__restrict__ sn,
                                    float sgn) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const int W4 = (3 * C) >> 2;
    if (g >= rows * W4) return;
    const int r = g / W4, col = (g - r * W4) * 4;
    float4 v = x[g];
    const int d = col % D;
    if (col < 2 * C && d < R) {
        const int half = R >> 1, t = r % T;
        const bool lo = d < half;
        const int i = lo ? d : d - half;
        const float4 q = x[lo ? g + (half >> 2) : g - (half >> 2)];
        const float4 c = *reinterpret_cast<const float4 *>(cs + t * half + i);
        const float4 s = *reinterpret_cast<const float4 *>(sn + t * half + i);
        // lo: v c - sgn q s; hi: v c + sgn q s -- rounded exactly as the scalar kernel is compiled
        // (fma(+-sgn q, s, round(v c))), so the two paths agree bitwise (tests/test_encoder_ops_gpu.py)
        const float m = lo ? -sgn : sgn;
        v = make_float4(__fmaf_rn(m * q.x, s.x, __fmul_rn(v.x, c.x)), __fmaf_rn(m * q.y, s.y, __fmul_rn(v.y, c.y)),
                        __fmaf_rn(m * q.z, s.z, __fmul_rn(v.z, c.z)), __fmaf_rn(m * q.w, s.w, __fmul_rn(v.w, c.w)));
    }
    y[g] = v;
}

}  // namespace

extern "C" {

int mtts_rope_qk(const float *x, float *y, int32_t rows, int32_t T, int32_t C, int32_t H, int32_t rope_dims,
                 const float *cos_t, const float *sin_t, int32_t inverse, void *hip_stream) {
    MTTS_CHECK_ARG(x && y && cos_t && sin_t && x != y, "rope_qk: null or aliased pointer");
    MTTS_CHECK_ARG(rows >= 0 && T >= 1 && rows % T == 0 && H >= 1 && C % H == 0 && rope_dims % 2 == 0 &&
                       rope_dims >= 0 && rope_dims <= C / H,
                   "rope_qk: bad shape");
    const int64_t n = (int64_t)rows * 3 * C;
    if (n == 0) return MTTS_OK;
    const int D = C / H;
    const bool al = ((uintptr_t)x | (uintptr_t)y | (uintptr_t)cos_t | (uintptr_t)sin_t) % 16 == 0;
    static const bool scalar_only = [] { const char *e = getenv("MTTS_ROPE_SCALAR"); return e && e[0] == '1'; }();
    if (!scalar_only && al && C % 4 == 0 && D % 4 == 0 && rope_dims % 8 == 0 && n / 4 < INT32_MAX) {
        const int64_t n4 = n / 4;
        hipLaunchKernelGGL(rope_qk_vec4_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0,
                           static_cast<hipStream_t>(hip_stream), reinterpret_cast<const float4 *>(x),
                           reinterpret_cast<float4 *>(y), rows, T, C, D, rope_dims, cos_t, sin_t,
                           inverse ? -1.f : 1.f);
        return mtts::check_launch("rope_qk_vec4_kernel");
    }
    hipLaunchKernelGGL(rope_qk_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(hip_stream), x, y, rows, T, C, C / H, rope_dims, cos_t, sin_t,
                       inverse ? -1.f : 1.f);
    return mtts::check_launch("rope_qk_kernel");
}


int mtts_attention_fwd(const mtts_attn_args *p, int32_t precision, void *hip_stream) {
    if (int rc = check_args(p, precision)) return rc;
    if (p->B == 0 || p->T == 0) return MTTS_OK;
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    return precision == MTTS_PREC_BF16 ? fwd_dispatch<true>(*p, st) : fwd_dispatch<false>(*p, st);
}

size_t mtts_attention_bwd_workspace_size(int32_t B, int32_t T, int32_t H) {
    return mtts::align_up((size_t)B * H * T * sizeof(float), 256);
}

int mtts_attention_bwd(const mtts_attn_args *p, const mtts_attn_grads *g, int32_t precision, void *workspace,
                       size_t workspace_bytes, void *hip_stream) {
    if (int rc = check_args(p, precision)) return rc;
    MTTS_CHECK_ARG(g && g->dout && g->dq && g->dk && g->dv, "attention_bwd: null gradient tensor");
    MTTS_CHECK_ARG(g->lddo % 4 == 0 && g->ldd % 4 == 0 && g->lddo >= p->H * p->D && g->ldd >= p->H * p->D,
                   "attention_bwd: gradient row strides must be multiples of 4 and cover H*D");
    MTTS_CHECK_ARG(aligned16(g->dout) && aligned16(g->dq) && aligned16(g->dk) && aligned16(g->dv),
                   "attention_bwd: gradients must be 16-byte aligned");
    if (p->B == 0 || p->T == 0) return MTTS_OK;
    if (workspace_bytes < mtts_attention_bwd_workspace_size(p->B, p->T, p->H) || !workspace)
        return mtts::fail(MTTS_ERR_WORKSPACE, "attention_bwd: workspace too small");
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    float *Drow = static_cast<float *>(workspace);
    return precision == MTTS_PREC_BF16 ? bwd_dispatch<true>(*p, *g, Drow, st) : bwd_dispatch<false>(*p, *g, Drow, st);
}

}  // extern "C"
