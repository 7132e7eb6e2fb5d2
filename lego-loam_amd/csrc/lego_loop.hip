// lego_loop.hip — mapOptimization's loop closure (performLoopClosure,
// mapOptmization.cpp:875-945) on gfx950, over the device keyframe store the
// mapping step maintains (lego_mo.hip):
//   k_lc_detect   detectLoopClosure (:814-872): the keyframe with the smallest
//                 (distance, index) among those within historyKeyframeSearchRadius
//                 of the robot and more than 30 s old — the first such hit of the
//                 reference's distance-sorted radius search — and the gather plan
//                 of the latest keyframe and the +-25 around it;
//   k_lc_gather   transformPointCloud (:577-606) of the planned keyframe clouds,
//                 one workgroup per (keyframe, cloud);
//   k_lc_compact  the latest keyframe's points with int(intensity) >= 0, in order;
//   VoxelGrid 0.4 and a 1 m hashed-cell index over the history cloud (lego_mo.hip);
//   k_icp_corr    pcl::IterativeClosestPoint's correspondences: the exact nearest
//                 history point of every source point, one wave per point (27
//                 cells, else the whole cloud), kept within 100 m;
//   k_icp_solve   umeyama over the correspondences (double reductions, the
//                 shared JacobiSVD restatement), final = T * final, the
//                 DefaultConvergenceCriteria test; one workgroup;
//   k_icp_apply   the source cloud moved by T (the next iteration's input);
//   k_icp_fit*    getFitnessScore: the nearest-neighbour distances of the source
//                 under the final transformation, averaged in double.
// The host runs the iterations (a completion flag read back every few) and
// turns the final transformation into the loop constraint (lego_icp.h).
#include <cfloat>
#include <climits>

#include "lego_device.h"
#include "lego_icp.h"
#include "lego_kernels.h"
#include "lego_mo.h"

namespace lego {

constexpr double kLcRadius = 7.0;   // historyKeyframeSearchRadius, utility.h:132
constexpr double kLcTime = 30.0;    // detectLoopClosure :830
constexpr int kLcHist = 25;         // historyKeyframeSearchNum, utility.h:133
constexpr float kIcpMaxDist2 = 100.0f * 100.0f;  // setMaxCorrespondenceDistance(100)

__device__ __forceinline__ float4 kf_xform(const float* pose, float4 p) {  // transformPointCloud :577-606
  const float ctRoll = lego_cosf(pose[3]), stRoll = lego_sinf(pose[3]);
  const float ctPitch = lego_cosf(pose[4]), stPitch = lego_sinf(pose[4]);
  const float ctYaw = lego_cosf(pose[5]), stYaw = lego_sinf(pose[5]);
  const float x1 = ctYaw * p.x - stYaw * p.y;
  const float y1 = stYaw * p.x + ctYaw * p.y;
  const float z1 = p.z;
  const float x2 = x1;
  const float y2 = ctRoll * y1 - stRoll * z1;
  const float z2 = stRoll * y1 + ctRoll * z1;
  return make_float4(ctPitch * x2 + stPitch * z2 + pose[0], y2 + pose[1], -stPitch * x2 + ctPitch * z2 + pose[2], p.w);
}

// ---------------------------------------------------------------- detection
__global__ void __launch_bounds__(1024) k_lc_detect(MoKeyframes kf, double tnow, LcState* ls) {
  __shared__ unsigned long long best[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int K = kf.meta[KF_K];
  const float* robot = kf.robot + 3;  // currentRobotPosPoint (saveKeyFramesAndFactor :1355-1357)
  unsigned long long key = ~0ull;
  for (int i = tid; i < K; i += blockDim.x) {
    const float4 p = kf.pos3[i];
    float d = 0.f, e;
    e = robot[0] - p.x; d += e * e;
    e = robot[1] - p.y; d += e * e;
    e = robot[2] - p.z; d += e * e;
    if ((double)d <= kLcRadius * kLcRadius && fabs(kf.time[i] - tnow) > kLcTime) {
      const unsigned long long k = ((unsigned long long)__float_as_uint(d) << 32) | (unsigned)i;
      key = k < key ? k : key;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long y = __shfl_xor(key, o, 64);
    key = y < key ? y : key;
  }
  if (lane == 0) best[wave] = key;
  __syncthreads();
  if (tid != 0) return;
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) key = best[w] < key ? best[w] : key;
  LcState s = {};
  s.K = K;
  s.closest = key == ~0ull ? -1 : (int)(unsigned)key;
  s.latest = K - 1;
  s.detected = s.closest >= 0 ? 1 : 0;
  if (s.detected) {
    // the latest keyframe's corner and surf clouds, then the +-25 history keyframes'
    int n = 0, os = 0, ot = 0;
    for (int c = 0; c < 2; ++c) {
      const int* sg = kf.seg + 6 * s.latest;
      s.plan[n][0] = s.latest; s.plan[n][1] = sg[2 * c]; s.plan[n][2] = sg[2 * c + 1]; s.plan[n][3] = os;
      os += sg[2 * c + 1];
      ++n;
    }
    s.nPlanSrc = n;
    for (int j = -kLcHist; j <= kLcHist; ++j) {
      const int id = s.closest + j;
      if (id < 0 || id > s.latest) continue;
      const int* sg = kf.seg + 6 * id;
      for (int c = 0; c < 2; ++c) {
        s.plan[n][0] = id; s.plan[n][1] = sg[2 * c]; s.plan[n][2] = sg[2 * c + 1]; s.plan[n][3] = ot;
        ot += sg[2 * c + 1];
        ++n;
      }
    }
    s.nPlan = n;
    s.nSrcRaw = os;
    s.nTgtRaw = ot;
  }
  *ls = s;
}

__global__ void k_lc_gather(MoKeyframes kf, const LcState* ls, float4* srcRaw, float4* tgtRaw) {
  const int b = blockIdx.x;
  if (b >= ls->nPlan) return;
  const int key = ls->plan[b][0], off = ls->plan[b][1], n = ls->plan[b][2], out = ls->plan[b][3];
  float4* dst = (b < ls->nPlanSrc ? srcRaw : tgtRaw) + out;
  const float* pose = kf.pose6 + 6 * key;
  for (int j = threadIdx.x; j < n; j += blockDim.x) dst[j] = kf_xform(pose, kf.arena[off + j]);
}

// hahaCloud (:843-849): the points with int(intensity) >= 0, order kept
__global__ void __launch_bounds__(1024) k_lc_compact(const float4* srcRaw, LcState* ls, float4* src, float4* cur) {
  __shared__ int wcnt[16];
  __shared__ int base;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = ls->nSrcRaw;
  if (tid == 0) base = 0;
  __syncthreads();
  for (int c0 = 0; c0 < n; c0 += blockDim.x) {
    const int i = c0 + tid;
    float4 p = make_float4(0, 0, 0, -1);
    if (i < n) p = srcRaw[i];
    const bool keep = i < n && (int)p.w >= 0;
    const unsigned long long m = __ballot(keep);
    const int rank = __popcll(m & ((1ull << lane) - 1));
    if (lane == 0) wcnt[wave] = __popcll(m);
    __syncthreads();
    int off = base;
    for (int w = 0; w < wave; ++w) off += wcnt[w];
    if (keep) {
      src[off + rank] = p;
      cur[off + rank] = p;
    }
    __syncthreads();
    if (tid == 0)
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) base += wcnt[w];
    __syncthreads();
  }
  if (tid == 0) ls->nSrc = base;
}

// ---------------------------------------------------------------- nearest neighbour
__device__ __forceinline__ unsigned lc_cell_hash(int ix, int iy, int iz) {  // = lego_mo.hip's mo_cell_hash
  unsigned long long k = ((unsigned long long)(unsigned)(ix + (1 << 20)) << 42) |
                         ((unsigned long long)(unsigned)(iy + (1 << 20)) << 21) |
                         (unsigned long long)(unsigned)(iz + (1 << 20));
  k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33;
  return (unsigned)k;
}
__device__ __forceinline__ float flann_d2q(float4 q, float4 p) {  // L2_Simple order ((0 + dx^2) + dy^2) + dz^2
  float r = 0.f, d;
  d = q.x - p.x; r += d * d;
  d = q.y - p.y; r += d * d;
  d = q.z - p.z; r += d * d;
  return r;
}
__device__ __forceinline__ void lc_lex_min(float& d, int& i, float d2, int i2) {
  if (d2 < d || (d2 == d && i2 < i)) { d = d2; i = i2; }
}
__device__ __forceinline__ void lc_wave_lex_min(float& d, int& i) {  // (distance, index): two plain minima
  float dm = d;
  for (int o = 32; o > 0; o >>= 1) dm = fminf(dm, __shfl_xor(dm, o, 64));
  int im = d == dm ? i : INT_MAX;
  for (int o = 32; o > 0; o >>= 1) im = min(im, __shfl_xor(im, o, 64));
  d = dm;
  i = im;
}
// The exact nearest history point of q (KdTreeFLANN::nearestKSearch k = 1;
// ties -> lower index) by the calling wave: the 27 cells around q, accepted
// when the best distance is under the 1 m they cover; else every point.
__device__ __forceinline__ void nn1_wave(const MoIndex& ix, const float4* tgt, int nT, float4 q, float* od, int* oi) {
  const int g = threadIdx.x & 63;
  float bd = FLT_MAX;
  int bi = INT_MAX;
  if (g < 54) {
    const int cc = g % 27, half = g / 27;
    const int bx = (int)floorf(q.x) + cc % 3 - 1, by = (int)floorf(q.y) + (cc / 3) % 3 - 1,
              bz = (int)floorf(q.z) + cc / 9 - 1;
    const unsigned b = lc_cell_hash(bx, by, bz) & (unsigned)(ix.T - 1);
    const int lo = ix.begin[b], hi = ix.end[b];
    for (int t = lo + half; t < hi; t += 2) {
      const float4 p = ix.sorted[t];
      lc_lex_min(bd, bi, flann_d2q(q, p), __float_as_int(p.w));
    }
  }
  lc_wave_lex_min(bd, bi);
  if (!(bd < 0.99999f)) {
    bd = FLT_MAX;
    bi = INT_MAX;
    for (int j = g; j < nT; j += 64) lc_lex_min(bd, bi, flann_d2q(q, tgt[j]), j);
    lc_wave_lex_min(bd, bi);
  }
  *od = bd;
  *oi = bi == INT_MAX ? -1 : bi;
}

// ---------------------------------------------------------------- ICP
// mode 0: correspondences of the current source (within 100 m); mode 1: the
// fitness distances of the original source moved by the final transformation
__global__ void k_icp_corr(MoIndex ix, const float4* tgt, const float4* src, const float4* cur, LcState* ls,
                           int* cIdx, float* cD, int mode) {
  if (mode == 0 && ls->done) return;
  const int nS = ls->nSrc, nT = ls->nTgt;
  const int waves = (gridDim.x * blockDim.x) >> 6;
  for (int q = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; q < nS; q += waves) {
    float4 p;
    if (mode == 0) {
      p = cur[q];
    } else {
      p = src[q];
      float x, y, z;
      xform_point(&ls->fin[0][0], p.x, p.y, p.z, &x, &y, &z);
      p.x = x; p.y = y; p.z = z;
    }
    float d;
    int i;
    nn1_wave(ix, tgt, nT, p, &d, &i);
    if ((threadIdx.x & 63) == 0) {
      const bool ok = i >= 0 && (mode == 1 || !(d > kIcpMaxDist2));
      cIdx[q] = ok ? i : -1;
      cD[q] = d;
    }
  }
}

// Block sum of N doubles, every thread gets the totals (fixed tree:
// butterfly within the wave, waves in order).
template <int N>
__device__ __forceinline__ void lc_block_sum(double (&v)[N], double* red /*[16 * N]*/) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < N; ++k)
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < N; ++k) red[wave * N + k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k) {
    double s = 0;
    for (int w = 0; w < nw; ++w) s += red[w * N + k];
    v[k] = s;
  }
  __syncthreads();
}

// umeyama (TransformationEstimationSVD) + final = T * final + hasConverged
__global__ void __launch_bounds__(1024) k_icp_solve(const float4* tgt, const float4* cur, LcState* ls, const int* cIdx,
                                                     const float* cD) {
  __shared__ double red[16 * 10];
  if (ls->done) return;
  const int tid = threadIdx.x, nS = ls->nSrc;
  double a[7] = {0, 0, 0, 0, 0, 0, 0};  // src xyz, tgt xyz, count
  for (int i = tid; i < nS; i += blockDim.x) {
    const int j = cIdx[i];
    if (j < 0) continue;
    const float4 s = cur[i], t = tgt[j];
    a[0] += s.x; a[1] += s.y; a[2] += s.z;
    a[3] += t.x; a[4] += t.y; a[5] += t.z;
    a[6] += 1.0;
  }
  lc_block_sum<7>(a, red);
  const int n = (int)a[6];
  if (n < 3) {  // min_number_correspondences_: converged_ = false, break
    if (tid == 0) { ls->done = 1; ls->converged = 0; }
    return;
  }
  const float one_over_n = 1.0f / (float)n;
  const float sm[3] = {(float)a[0] * one_over_n, (float)a[1] * one_over_n, (float)a[2] * one_over_n};
  const float dm[3] = {(float)a[3] * one_over_n, (float)a[4] * one_over_n, (float)a[5] * one_over_n};
  double b[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // sigma (row-major) + the squared distances
  for (int i = tid; i < nS; i += blockDim.x) {
    const int j = cIdx[i];
    if (j < 0) continue;
    const float4 s = cur[i], t = tgt[j];
    const float s3[3] = {s.x - sm[0], s.y - sm[1], s.z - sm[2]};
    const float d3[3] = {t.x - dm[0], t.y - dm[1], t.z - dm[2]};
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) b[3 * r + c] += (double)d3[r] * (double)s3[c];
    b[9] += cD[i];
  }
  lc_block_sum<10>(b, red);
  if (tid != 0) return;
  float sigma[3][3], T[4][4];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) sigma[r][c] = (float)b[3 * r + c] * one_over_n;
  umeyama_finish(sm, dm, sigma, T);
  float nf[4][4];
  mat4_mul(T, ls->fin, nf);
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) { ls->fin[r][c] = nf[r][c]; ls->T[r][c] = T[r][c]; }
  ls->iterations += 1;
  IcpCriteria crit = ls->crit;
  const bool conv = icp_converged(crit, ls->iterations, T, b[9] / (double)n);
  ls->crit = crit;
  ls->converged = conv ? 1 : 0;
  ls->done = conv ? 1 : 0;  // the last transform is not applied: nothing reads the moved cloud after
}

__global__ void k_icp_apply(float4* cur, LcState* ls) {
  if (ls->done) return;
  const int n = ls->nSrc;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    float4 p = cur[i];
    float x, y, z;
    xform_point(&ls->T[0][0], p.x, p.y, p.z, &x, &y, &z);
    cur[i] = make_float4(x, y, z, p.w);
  }
}

__global__ void __launch_bounds__(1024) k_icp_fitsum(LcState* ls, const int* cIdx, const float* cD) {
  __shared__ double red[16 * 2];
  double a[2] = {0, 0};
  for (int i = threadIdx.x; i < ls->nSrc; i += blockDim.x)
    if (cIdx[i] >= 0) { a[0] += cD[i]; a[1] += 1.0; }
  lc_block_sum<2>(a, red);
  if (threadIdx.x == 0) {
    ls->nFit = (int)a[1];
    ls->fitness = a[1] > 0 ? a[0] / a[1] : DBL_MAX;
  }
}

__global__ void k_lc_init(LcState* ls) {
  ls->iterations = 0;
  ls->converged = 0;
  ls->done = 0;
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) ls->fin[r][c] = r == c ? 1.0f : 0.0f;
  ls->crit = icp_criteria(100, 1e-6, 1e-6);  // setMaximumIterations / setTransformationEpsilon / setEuclideanFitnessEpsilon
}

static int lc_grid(int n, int per = 256) {
  int g = (n + per - 1) / per;
  return g < 1 ? 1 : (g > 4096 ? 4096 : g);
}

int mo_loop_closure_device(MoDev& m, LcDev& lc, double tnow, LcState* hostState, hipStream_t s) {
  k_lc_detect<<<1, 1024, 0, s>>>(m.kf, tnow, lc.st);
  if (hipMemcpyAsync(hostState, lc.st, sizeof(LcState), hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
  if (hipStreamSynchronize(s) != hipSuccess) return -1;
  if (!hostState->detected) return 0;
  if (hostState->nSrcRaw > lc.cap || hostState->nTgtRaw > lc.cap || hostState->nTgtRaw > m.vg.cap) return MO_E_MAP_CAP;
  k_lc_gather<<<hostState->nPlan, 256, 0, s>>>(m.kf, lc.st, lc.srcRaw, lc.tgtRaw);
  k_lc_compact<<<1, 1024, 0, s>>>(lc.srcRaw, lc.st, lc.src, lc.cur);
  if (voxel_grid_device(lc.tgtRaw, hostState->nTgtRaw, nullptr, 0.4f, lc.tgt, &lc.st->nTgt, m.vg, s)) return -1;
  if (index_build_device(lc.tgt, hostState->nTgtRaw, &lc.st->nTgt, lc.ix, m.vg, s)) return -1;
  k_lc_init<<<1, 1, 0, s>>>(lc.st);
  const int nS = hostState->nSrcRaw;  // upper bound of the compacted source
  const int corrBlocks = lc_grid(nS, 4);  // 256 threads = 4 waves per block, one wave per point
  for (int it = 0; it < 100;) {
    for (int k = 0; k < 4 && it < 100; ++k, ++it) {  // done-gated: extra launches return at once
      k_icp_corr<<<corrBlocks, 256, 0, s>>>(lc.ix, lc.tgt, lc.src, lc.cur, lc.st, lc.cIdx, lc.cD, 0);
      k_icp_solve<<<1, 1024, 0, s>>>(lc.tgt, lc.cur, lc.st, lc.cIdx, lc.cD);
      k_icp_apply<<<lc_grid(nS), 256, 0, s>>>(lc.cur, lc.st);
    }
    if (hipMemcpyAsync(&hostState->done, &lc.st->done, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess)
      return -1;
    if (hipStreamSynchronize(s) != hipSuccess) return -1;
    if (hostState->done) break;
  }
  k_icp_corr<<<corrBlocks, 256, 0, s>>>(lc.ix, lc.tgt, lc.src, lc.cur, lc.st, lc.cIdx, lc.cD, 1);
  k_icp_fitsum<<<1, 1024, 0, s>>>(lc.st, lc.cIdx, lc.cD);
  if (hipMemcpyAsync(hostState, lc.st, sizeof(LcState), hipMemcpyDeviceToHost, s) != hipSuccess) return -1;
  if (hipStreamSynchronize(s) != hipSuccess) return -1;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lego
