// microbenchmark: the corner LM row loop of lm_loop (one query per lane, 192 queries)
#include "../../lego-loam_amd/csrc/lego_odom.hip"
using namespace lego;
template <int MODE>
__global__ void __launch_bounds__(512) krow(const float4* gq, const float4* glast, const int* gqi, double* o,
                                            long long* t, int iters, int nQ) {
  __shared__ float4 qp[384], last[2048];
  __shared__ int qi[3 * 384];
  const int tid = threadIdx.x;
  for (int i = tid; i < nQ; i += 512) { qp[i] = gq[i]; qi[i] = gqi[i]; qi[384 + i] = gqi[384 + i]; }
  for (int i = tid; i < 2048; i += 512) last[i] = glast[i];
  __syncthreads();
  float tc[6] = {0.01f, 0.02f, -0.015f, 0.1f, 0.05f, 0.2f};
  FixTrig fix; fix.have = false;
  double tot = 0;
  const int qs = 384;
  const bool surf = false;
  long long t0 = wall_clock64();
  for (int it = 0; it < iters; ++it) {
    float trig;
    { const int l = tid & 63; const float a = tc[l % 3]; trig = l < 3 ? lego_sinf(a) : lego_cosf(a); }
    const float srx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(trig), 0));
    const float sry = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(trig), 1));
    const float srz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(trig), 2));
    const float crx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(trig), 3));
    const float cry = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(trig), 4));
    const float crz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(trig), 5));
    const float tx = tc[3], ty = tc[4], tz = tc[5];
    double acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int mloc = 0;
    const int qstep = MODE == 5 ? 64 : 512;  // mode 5: wave 0 takes every row (3 per lane)
    for (int q = (MODE == 5 && tid >= 64) ? nQ : tid; q < nQ; q += qstep) {
      const float4 po = qp[q];
      float4 sel;
      if (MODE == 2) sel = to_start_t(po, start_s(po), tc, 1.f, 0.f, 1.f, 0.f, 1.f, 0.f);
      else sel = q == tid ? to_start_fix(po, tc, surf, fix) : to_start(po, tc);
      const int i1 = qi[q], i2 = qi[qs + q];
      float4 cf; bool ok = false;
      if (i2 >= 0) {
        const float4 t1 = last[i1], t2 = last[i2];
        const float x0 = sel.x, y0 = sel.y, z0 = sel.z;
        const float x1 = t1.x, y1 = t1.y, z1 = t1.z, x2 = t2.x, y2 = t2.y, z2 = t2.z;
        const float m11 = ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1));
        const float m22 = ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1));
        const float m33 = ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1));
        const float a012 = __builtin_sqrtf(m11 * m11 + m22 * m22 + m33 * m33);
        const float l12 = __builtin_sqrtf((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
        float la, lb, lc, ld2;
        if (MODE == 3) {
          la = ((y1 - y2) * m11 + (z1 - z2) * m22) * a012 * l12;
          lb = -((x1 - x2) * m11 - (z1 - z2) * m33) * a012 * l12;
          lc = -((x1 - x2) * m22 + (y1 - y2) * m33) * a012 * l12;
          ld2 = a012 * l12;
        } else {
          la = ((y1 - y2) * m11 + (z1 - z2) * m22) / a012 / l12;
          lb = -((x1 - x2) * m11 - (z1 - z2) * m33) / a012 / l12;
          lc = -((x1 - x2) * m22 + (y1 - y2) * m33) / a012 / l12;
          ld2 = a012 / l12;
        }
        float s = 1;
        if (it >= 5) s = (float)(1 - 1.8 * (double)lfabsf(ld2));
        if ((double)s > 0.1 && ld2 != 0) { ok = true; cf = make_float4(s * la, s * lb, s * lc, s * ld2); }
      }
      if (ok) {
        const float b1 = -crz * sry - cry * srx * srz, b2 = cry * crz * srx - sry * srz, b3 = crx * cry;
        const float b4 = tx * -b1 + ty * -b2 + tz * b3;
        const float b5 = cry * crz - srx * sry * srz, b6 = cry * srz + crz * srx * sry, b7 = crx * sry;
        const float b8 = tz * b7 - ty * b6 - tx * b5;
        const float c5 = crx * srz;
        const float a0 = (b1 * po.x + b2 * po.y - b3 * po.z + b4) * cf.x + (b5 * po.x + b6 * po.y - b7 * po.z + b8) * cf.z;
        const float a1 = -b5 * cf.x + c5 * cf.y + b1 * cf.z;
        const float a2 = b7 * cf.x - srx * cf.y - b3 * cf.z;
        const float bb = (float)(-0.05 * (double)cf.w);
        const double d0 = a0, d1 = a1, d2 = a2, db = bb;
        if (MODE == 1) {
          acc[0] = __builtin_fma(d0, d0, acc[0]); acc[1] = __builtin_fma(d0, d1, acc[1]); acc[2] = __builtin_fma(d0, d2, acc[2]);
          acc[3] = __builtin_fma(d1, d1, acc[3]); acc[4] = __builtin_fma(d1, d2, acc[4]); acc[5] = __builtin_fma(d2, d2, acc[5]);
          acc[6] = __builtin_fma(d0, db, acc[6]); acc[7] = __builtin_fma(d1, db, acc[7]); acc[8] = __builtin_fma(d2, db, acc[8]);
        } else {
          acc[0] += d0 * d0; acc[1] += d0 * d1; acc[2] += d0 * d2;
          acc[3] += d1 * d1; acc[4] += d1 * d2; acc[5] += d2 * d2;
          acc[6] += d0 * db; acc[7] += d1 * db; acc[8] += d2 * db;
        }
        mloc++;
      }
    }
    if (MODE == 4) __syncthreads();
    if (MODE == 5 && tid < 64) {  // the wave's DPP reduction, no barrier
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const double r = row_sum_f64(acc[k]);
        acc[k] = ((rdlane_f64(r, 0) + rdlane_f64(r, 16)) + rdlane_f64(r, 32)) + rdlane_f64(r, 48);
      }
    }
    for (int k = 0; k < 9; ++k) tot += acc[k];
    tot += mloc;
    tc[1] += (float)(acc[0] * 1e-30);  // keep the loop honest; ry changes each iteration
  }
  long long t1 = wall_clock64();
  if (tid == 0) { *t = t1 - t0; }
  o[tid] = tot;
}
int main() {
  const int nQ = 192;
  float4 hq[384], hl[2048]; int hqi[3 * 384];
  srand(1);
  auto R = [] { return (float)rand() / RAND_MAX * 20.f - 10.f; };
  for (int i = 0; i < 2048; ++i) hl[i] = make_float4(R(), R(), R() * 0.2f, (float)(i % 16));
  for (int i = 0; i < 384; ++i) { hq[i] = make_float4(R(), R(), R() * 0.2f, (float)(i % 16) + 0.01f * (i % 97));
    hqi[i] = rand() % 2048; hqi[384 + i] = rand() % 2048; hqi[768 + i] = -1; }
  float4 *dq, *dl; int* dqi; double* o; long long* t;
  (void)hipMalloc(&dq, sizeof hq); (void)hipMalloc(&dl, sizeof hl); (void)hipMalloc(&dqi, sizeof hqi);
  (void)hipMalloc(&o, 512 * 8); (void)hipMalloc(&t, 8);
  (void)hipMemcpy(dq, hq, sizeof hq, hipMemcpyHostToDevice); (void)hipMemcpy(dl, hl, sizeof hl, hipMemcpyHostToDevice);
  (void)hipMemcpy(dqi, hqi, sizeof hqi, hipMemcpyHostToDevice);
  const char* nm[6] = {"current", "fma acc", "no trig", "no div", "current+barrier", "one wave + DPP sum"};
  for (int mode = 0; mode < 6; ++mode) {
    long long ht = 0;
    for (int rep = 0; rep < 2; ++rep) {
      const int iters = 5000;
      switch (mode) {
        case 0: krow<0><<<1, 512>>>(dq, dl, dqi, o, t, iters, nQ); break;
        case 1: krow<1><<<1, 512>>>(dq, dl, dqi, o, t, iters, nQ); break;
        case 2: krow<2><<<1, 512>>>(dq, dl, dqi, o, t, iters, nQ); break;
        case 3: krow<3><<<1, 512>>>(dq, dl, dqi, o, t, iters, nQ); break;
        case 4: krow<4><<<1, 512>>>(dq, dl, dqi, o, t, iters, nQ); break;
        case 5: krow<5><<<1, 512>>>(dq, dl, dqi, o, t, iters, nQ); break;
      }
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(&ht, t, 8, hipMemcpyDeviceToHost);
    }
    printf("%-16s: %.3f us per iteration\n", nm[mode], ht / 100.0 / 5000);
  }
  return 0;
}
