// Batched fixed-order partial-sum reductions for the parameter gradients (gfx950).
//
// The weight-gradient GEMM splits its token range into fp32 slabs, and the LayerNorm / GroupNorm
// backwards leave per-block gamma/beta partials; each used to end in its own small reduce launch
// (~120 launches per training step, ~1.1 ms of mostly tail).  A job here is
//     out[map(i)] (+)= sum_{s < splits} part[s*stride + i],  i < n        (mtts_decoder.h)
// and one launch runs up to kJobs jobs side by side: the grid is the concatenation of every job's
// blocks (blockIdx -> job by a scan over the batch's first-block table, wave-uniform).  A block owns
// `gpb` float4 groups of one job; its 256 threads are 256/gpb slices that take interleaved slabs (4
// loads in flight per lane), and the slice sums are added through LDS in a fixed order -- the result
// is bitwise reproducible.  Long, narrow jobs (the norm partials: ~500 slabs of 256 columns) use 16
// groups x 16 slices per block; wide ones (weight gradients) 64 groups x 4 slices.
//
// mtts_colsum: column sums of a tall matrix as per-128-row-chunk partials (one launch) + one such job (the
// transposed conv's bias gradient, decoder.py:112), fixed order like the rest.
//
// Deferral (mtts_defer_reductions) queues the jobs of a whole backward pass and mtts_flush_reductions
// runs them in one batched launch; the queue is process-wide because autograd calls the backward
// entry points from its own thread.  The weight-gradient GEMMs themselves are deferred too
// (conv_gemm.hip, MTTS_DEFER_WGRAD): a flush first launches them batched, then their slab sums.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <vector>

#include "mtts_common.h"
#include "mtts_decoder.h"

namespace {

constexpr int kJobs = 32;
constexpr int kThreads = 256;

struct ReduceBatch {
    mtts_reduce_job job[kJobs];
    int32_t first[kJobs + 1];  // first block of each job; first[njobs] = grid size
    int32_t gpb[kJobs];        // float4 groups per block: 16 or 64
    int32_t vec[kJobs];        // float4 loads (n % 4 == 0, stride % 4 == 0, 16-byte aligned part)
    int32_t njobs;
};

__device__ __forceinline__ void add4(float4 &a, const float4 &b) {
    a.x += b.x;
    a.y += b.y;
    a.z += b.z;
    a.w += b.w;
}

__global__ __launch_bounds__(kThreads) void reduce_partials_kernel(const ReduceBatch rb) {
    __shared__ float4 red[kThreads];
    int j = 0;
    while (j + 1 < rb.njobs && (int)blockIdx.x >= rb.first[j + 1]) ++j;
    const mtts_reduce_job &J = rb.job[j];
    const int gpb = rb.gpb[j], slices = kThreads / gpb;
    const int t = threadIdx.x % gpb, sl = threadIdx.x / gpb;
    const int64_t q = (int64_t)(blockIdx.x - rb.first[j]) * gpb + t;  // float4 group of this thread
    const int64_t e0 = 4 * q;
    const bool on = e0 < J.n;
    const bool vec = rb.vec[j] != 0;
    auto load = [&](int s) -> float4 {
        const float *src = J.part + (int64_t)s * J.stride + e0;
        if (vec) return on ? *reinterpret_cast<const float4 *>(src) : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e0 < J.n) v.x = src[0];
        if (e0 + 1 < J.n) v.y = src[1];
        if (e0 + 2 < J.n) v.z = src[2];
        if (e0 + 3 < J.n) v.w = src[3];
        return v;
    };
    float4 a[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) a[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    int s = sl;
    for (; s + 3 * slices < J.splits; s += 4 * slices) {
        float4 v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = load(s + c * slices);
#pragma unroll
        for (int c = 0; c < 4; ++c) add4(a[c], v[c]);
    }
#pragma unroll
    for (int c = 0; c < 3; ++c)
        if (s + c * slices < J.splits) add4(a[c], load(s + c * slices));
    add4(a[0], a[1]);
    add4(a[2], a[3]);
    add4(a[0], a[2]);
    red[threadIdx.x] = a[0];
    __syncthreads();
    if (sl != 0 || !on) return;
    float4 r = red[t];
    for (int i = 1; i < slices; ++i) add4(r, red[i * gpb + t]);
    const float rv[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int64_t i = e0 + e;
        if (i >= J.n) break;
        int64_t idx = i;
        if (J.cols > 0) {
            const int64_t row = i / J.cols;
            const int k = (int)(i - row * J.cols), jj = k / J.cin, c = k - jj * J.cin;
            idx = row * J.sr + c * J.sc + jj * J.sj;
        }
        J.out[idx] = J.accumulate ? J.out[idx] + rv[e] : rv[e];
    }
}

int launch_jobs(const mtts_reduce_job *jobs, int njobs, hipStream_t st) {
    for (int base = 0; base < njobs; base += kJobs) {
        const int n = njobs - base < kJobs ? njobs - base : kJobs;
        ReduceBatch rb;
        int64_t blocks = 0;
        int used = 0;
        for (int i = 0; i < n; ++i) {
            const mtts_reduce_job &J = jobs[base + i];
            if (J.n <= 0) continue;
            const int64_t groups = (J.n + 3) / 4;
            const int gpb = (J.splits >= 64 && groups <= 1024) ? 16 : 64;
            rb.job[used] = J;
            rb.first[used] = (int32_t)blocks;
            rb.gpb[used] = gpb;
            rb.vec[used] = (J.n % 4 == 0 && J.stride % 4 == 0 && (reinterpret_cast<uintptr_t>(J.part) & 15) == 0);
            blocks += (groups + gpb - 1) / gpb;
            ++used;
        }
        if (used == 0) continue;
        if (blocks > INT32_MAX) return mtts::fail(MTTS_ERR_SHAPE, "reduce_partials: too many blocks");
        rb.first[used] = (int32_t)blocks;
        rb.njobs = used;
        hipLaunchKernelGGL(reduce_partials_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, st, rb);
        if (int rc = mtts::check_launch("reduce_partials_kernel")) return rc;
    }
    return MTTS_OK;
}

int check_jobs(const mtts_reduce_job *jobs, int njobs) {
    MTTS_CHECK_ARG(njobs >= 0 && (jobs || njobs == 0), "reduce_partials: bad job list");
    for (int i = 0; i < njobs; ++i) {
        const mtts_reduce_job &J = jobs[i];
        MTTS_CHECK_ARG(J.n >= 0 && J.splits >= 1 && J.stride >= J.n, "reduce_partials: need splits >= 1, stride >= n");
        MTTS_CHECK_ARG(J.n == 0 || (J.part && J.out), "reduce_partials: null pointer");
        MTTS_CHECK_ARG(J.cols >= 0 && (J.cols == 0 || (J.cin > 0 && J.cols % J.cin == 0 && J.n % J.cols == 0)),
                       "reduce_partials: weight layout needs cin | cols | n");
    }
    return MTTS_OK;
}

constexpr int kColChunk = 128;

__global__ __launch_bounds__(256) void colsum_partials_kernel(const float *__restrict__ x, int64_t rows, int n, int ld,
                                                              float *__restrict__ part) {
    const int c = blockIdx.y * 256 + threadIdx.x;
    if (c >= n) return;
    const int64_t r0 = (int64_t)blockIdx.x * kColChunk;
    const int64_t r1 = r0 + kColChunk < rows ? r0 + kColChunk : rows;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;  // four chains, added in a fixed order
    int64_t r = r0;
    for (; r + 3 < r1; r += 4) {
        a0 += x[r * ld + c];
        a1 += x[(r + 1) * ld + c];
        a2 += x[(r + 2) * ld + c];
        a3 += x[(r + 3) * ld + c];
    }
    for (; r < r1; ++r) a0 += x[r * ld + c];
    part[(size_t)blockIdx.x * n + c] = (a0 + a1) + (a2 + a3);
}

std::mutex g_mu;
bool g_defer = false;
std::vector<mtts_reduce_job> g_queue;

}  // namespace

namespace mtts {
int submit_reductions(const mtts_reduce_job *jobs, int njobs, hipStream_t st) {
    if (int rc = check_jobs(jobs, njobs)) return rc;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (g_defer) {
            g_queue.insert(g_queue.end(), jobs, jobs + njobs);
            return MTTS_OK;
        }
    }
    return launch_jobs(jobs, njobs, st);
}

int queue_reductions(const mtts_reduce_job *jobs, int njobs) {
    if (int rc = check_jobs(jobs, njobs)) return rc;
    std::lock_guard<std::mutex> lk(g_mu);
    g_queue.insert(g_queue.end(), jobs, jobs + njobs);
    return MTTS_OK;
}

bool deferring() {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_defer;
}
}  // namespace mtts

extern "C" {

int mtts_reduce_partials(const mtts_reduce_job *jobs, int32_t njobs, void *hip_stream) {
    if (int rc = check_jobs(jobs, njobs)) return rc;
    return launch_jobs(jobs, njobs, static_cast<hipStream_t>(hip_stream));
}

void mtts_defer_reductions(int32_t on) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_defer = on != 0;
}

int32_t mtts_pending_reductions(void) {
    const int w = mtts::pending_wgrad_sums();  // the queued weight gradients' slab sums, still to come
    std::lock_guard<std::mutex> lk(g_mu);
    return (int32_t)g_queue.size() + w;
}

int mtts_flush_reductions(void *hip_stream) {
    // queued weight gradients first (batched launches); their slab sums join the queue
    if (int rc = mtts::flush_wgrads(static_cast<hipStream_t>(hip_stream))) return rc;
    std::vector<mtts_reduce_job> q;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        q.swap(g_queue);
    }
    return launch_jobs(q.data(), (int)q.size(), static_cast<hipStream_t>(hip_stream));
}

int mtts_colsum(const float *x, int64_t rows, int32_t n, int32_t ld, float *out, int32_t accumulate, float *workspace,
                size_t workspace_bytes, void *hip_stream) {
    MTTS_CHECK_ARG(x && out && rows >= 1 && n >= 1 && ld >= n, "colsum: bad args");
    const int64_t chunks = (rows + kColChunk - 1) / kColChunk;
    MTTS_CHECK_ARG(chunks <= INT32_MAX, "colsum: too many rows");
    if (!workspace || workspace_bytes < (size_t)chunks * n * sizeof(float))
        return mtts::fail(MTTS_ERR_WORKSPACE, "colsum: workspace too small");
    hipStream_t st = static_cast<hipStream_t>(hip_stream);
    hipLaunchKernelGGL(colsum_partials_kernel, dim3((unsigned)chunks, (n + 255) / 256), dim3(256), 0, st, x, rows, n, ld,
                       workspace);
    if (int rc = mtts::check_launch("colsum_partials_kernel")) return rc;
    mtts_reduce_job j = {};
    j.part = workspace;
    j.out = out;
    j.stride = n;
    j.n = n;
    j.splits = (int32_t)chunks;
    j.accumulate = accumulate;
    return mtts::submit_reductions(&j, 1, st);
}

size_t mtts_colsum_workspace_size(int64_t rows, int32_t n) {
    return rows < 1 || n < 1 ? 0 : (size_t)((rows + kColChunk - 1) / kColChunk) * n * sizeof(float);
}

void mtts_discard_reductions(void) {
    mtts::discard_wgrads();
    std::lock_guard<std::mutex> lk(g_mu);
    g_queue.clear();
}

}  // extern "C"
