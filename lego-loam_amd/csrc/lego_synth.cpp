// lego_synth.cpp — deterministic ray-cast lidar scenes (see include/lego_synth.h).
// Host-only data source for tests and bench; not part of the timed path.
#include "lego_synth.h"

#include <cmath>
#include <cstring>
#include <vector>

namespace {

inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() { s += 0x9e3779b97f4a7c15ULL; return mix64(s); }
  double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  double range(double a, double b) { return a + (b - a) * uni(); }
};
// stateless hash -> uniform / gaussian for per-ray noise (order independent)
inline double hash_uni(uint64_t key) {
  return (double)(mix64(key + 0x9e3779b97f4a7c15ULL) >> 11) * (1.0 / 9007199254740992.0);
}
inline double hash_gauss(uint64_t key) {
  double u1 = hash_uni(key * 2 + 1), u2 = hash_uni(key * 2 + 2);
  if (u1 < 1e-300) u1 = 1e-300;
  return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
}

struct Box { double cx, cy, cz, hx, hy, hz, yaw, c, s; };
struct Cyl { double cx, cy, r, z0, z1; };
struct Scene {
  double h, gx, gy;
  std::vector<Box> boxes;
  std::vector<Cyl> cyls;
};

// Ego trajectory: a circle of radius v/w (straight line if w == 0).
void ego_pose(const lego_synth_cfg& c, double t, double* px, double* py, double* yaw) {
  double v = c.speed_mps, w = c.yaw_rate_dps * M_PI / 180.0;
  if (std::fabs(w) < 1e-12) { *px = v * t; *py = 0; *yaw = 0; return; }
  double R = v / w;
  *yaw = w * t;
  *px = R * std::sin(w * t);
  *py = R * (1.0 - std::cos(w * t));
}

double dist_to_path(const lego_synth_cfg& c, double x, double y) {
  double v = c.speed_mps, w = c.yaw_rate_dps * M_PI / 180.0;
  if (std::fabs(w) < 1e-12) {
    if (x < 0) return std::hypot(x, y);
    return std::fabs(y);
  }
  double R = v / w;
  return std::fabs(std::hypot(x, y - R) - std::fabs(R));
}

Scene build_scene(const lego_synth_cfg& c) {
  Scene sc;
  Rng r(c.seed * 0x2545F4914F6CDD1DULL + 17);
  sc.h = c.mount_height;
  double tilt = c.ground_tilt_deg * M_PI / 180.0;
  sc.gx = std::tan(r.range(-tilt, tilt)) * 0.5;
  sc.gy = std::tan(r.range(-tilt, tilt)) * 0.5;
  auto ground_z = [&](double x, double y) { return -sc.h + sc.gx * x + sc.gy * y; };
  auto place = [&](double ext, double rmin, double rmax, double* x, double* y) {
    for (int tries = 0; tries < 1000; ++tries) {
      double a = r.range(-M_PI, M_PI), d = r.range(rmin, rmax);
      *x = d * std::cos(a);
      *y = d * std::sin(a);
      if (dist_to_path(c, *x, *y) > ext + 2.0 && std::hypot(*x, *y) > ext + 2.0) return;
    }
  };
  for (int i = 0; i < c.n_boxes; ++i) {
    Box b;
    b.hx = r.range(0.3, 3.0); b.hy = r.range(0.3, 3.0); b.hz = r.range(0.5, 3.0);
    place(std::hypot(b.hx, b.hy), 3.0, 60.0, &b.cx, &b.cy);
    b.yaw = r.range(-M_PI, M_PI); b.c = std::cos(b.yaw); b.s = std::sin(b.yaw);
    b.cz = ground_z(b.cx, b.cy) + b.hz - 0.2;
    sc.boxes.push_back(b);
  }
  for (int i = 0; i < c.n_cylinders; ++i) {
    Cyl y;
    y.r = r.range(0.1, 0.5);
    place(y.r, 3.0, 60.0, &y.cx, &y.cy);
    y.z0 = ground_z(y.cx, y.cy) - 0.2;
    y.z1 = y.z0 + r.range(2.0, 8.0);
    sc.cyls.push_back(y);
  }
  for (int i = 0; i < c.n_walls; ++i) {
    Box b;
    b.hx = r.range(10.0, 20.0); b.hy = 0.15; b.hz = r.range(1.5, 2.5);
    double a = r.range(-M_PI, M_PI), d = r.range(25.0, 40.0);
    b.cx = d * std::cos(a); b.cy = d * std::sin(a);
    b.yaw = a + M_PI / 2 + r.range(-0.3, 0.3);
    b.c = std::cos(b.yaw); b.s = std::sin(b.yaw);
    b.cz = ground_z(b.cx, b.cy) + b.hz - 0.2;
    sc.boxes.push_back(b);
  }
  return sc;
}

inline bool hit_box(const Box& b, const double o[3], const double d[3], double* t) {
  double ox = o[0] - b.cx, oy = o[1] - b.cy, oz = o[2] - b.cz;
  double lo[3] = {b.c * ox + b.s * oy, -b.s * ox + b.c * oy, oz};
  double ld[3] = {b.c * d[0] + b.s * d[1], -b.s * d[0] + b.c * d[1], d[2]};
  double hs[3] = {b.hx, b.hy, b.hz};
  double tn = -1e300, tf = 1e300;
  for (int k = 0; k < 3; ++k) {
    if (std::fabs(ld[k]) < 1e-15) {
      if (lo[k] < -hs[k] || lo[k] > hs[k]) return false;
      continue;
    }
    double t1 = (-hs[k] - lo[k]) / ld[k], t2 = (hs[k] - lo[k]) / ld[k];
    if (t1 > t2) { double tt = t1; t1 = t2; t2 = tt; }
    if (t1 > tn) tn = t1;
    if (t2 < tf) tf = t2;
    if (tn > tf) return false;
  }
  if (tn <= 1e-6) return false;
  *t = tn;
  return true;
}

inline bool hit_cyl(const Cyl& y, const double o[3], const double d[3], double* t) {
  double ox = o[0] - y.cx, oy = o[1] - y.cy;
  double a = d[0] * d[0] + d[1] * d[1];
  if (a < 1e-15) return false;
  double bq = 2 * (ox * d[0] + oy * d[1]);
  double cq = ox * ox + oy * oy - y.r * y.r;
  double disc = bq * bq - 4 * a * cq;
  if (disc < 0) return false;
  double tt = (-bq - std::sqrt(disc)) / (2 * a);
  if (tt <= 1e-6) return false;
  double z = o[2] + tt * d[2];
  if (z < y.z0 || z > y.z1) return false;
  *t = tt;
  return true;
}

double cast(const Scene& sc, const double o[3], const double d[3]) {
  double best = 1e300, t;
  double den = d[2] - sc.gx * d[0] - sc.gy * d[1];
  if (den < -1e-12) {
    t = (-sc.h + sc.gx * o[0] + sc.gy * o[1] - o[2]) / den;
    if (t > 0 && t < best) best = t;
  }
  for (const Box& b : sc.boxes)
    if (hit_box(b, o, d, &t) && t < best) best = t;
  for (const Cyl& y : sc.cyls)
    if (hit_cyl(y, o, d, &t) && t < best) best = t;
  return best;
}

}  // namespace

extern "C" int lego_synth_preset(const char* name, uint64_t seed, lego_synth_cfg* o) {
  if (!name || !o) return LEGO_E_ARG;
  std::memset(o, 0, sizeof(*o));
  o->mount_height = 0.6f;
  o->ground_tilt_deg = 3.0f;
  o->noise_sigma = 0.01f;
  o->dropout = 0.02f;
  o->max_range = 100.0f;
  o->dup_frac = 0.0f;
  o->azimuth_jitter = 0.2f;
  o->speed_mps = 1.0f;
  o->yaw_rate_dps = 5.0f;
  o->scan_period = 0.1f;
  o->n_boxes = 20;
  o->n_cylinders = 10;
  o->n_walls = 2;
  o->seed = seed;
  if (!std::strcmp(name, "VLP-16")) {
    o->n_scan = 16; o->horizon_scan = 1800; o->vert_min_deg = -15.f; o->vert_max_deg = 15.f;
  } else if (!std::strcmp(name, "HDL-64E")) {
    o->n_scan = 64; o->horizon_scan = 2048; o->vert_min_deg = -24.8f; o->vert_max_deg = 2.0f;
    o->mount_height = 1.73f;
  } else if (!std::strcmp(name, "VLS-128")) {
    o->n_scan = 128; o->horizon_scan = 1800; o->vert_min_deg = -25.f;
    o->vert_max_deg = -25.f + 0.3f * 127; o->mount_height = 1.2f;
  } else if (!std::strcmp(name, "HDL-32E")) {
    // utility.h:71-76: 41.33 deg over 32 rings from -30.67; the beams sit
    // 0.1 deg above the reference's row edges (as VLP-16's ang_bottom of
    // 15 + 0.1 does for its own), so the vertical-angle row of the
    // useCloudRing = false branch is the ring, not a float rounding away
    o->n_scan = 32; o->horizon_scan = 1800; o->vert_min_deg = -30.67f + 0.1f;
    o->vert_max_deg = -30.67f + 0.1f + 41.33f; o->mount_height = 1.5f;
  } else if (!std::strcmp(name, "OS1-16")) {  // utility.h:89-94: +-16.6 deg
    o->n_scan = 16; o->horizon_scan = 1024; o->vert_min_deg = -16.6f; o->vert_max_deg = 16.6f;
  } else if (!std::strcmp(name, "OS1-64")) {  // utility.h:97-102
    o->n_scan = 64; o->horizon_scan = 1024; o->vert_min_deg = -16.6f; o->vert_max_deg = 16.6f;
    o->mount_height = 1.2f;
  } else {
    return LEGO_E_ARG;
  }
  return LEGO_OK;
}

extern "C" int32_t lego_synth_max_points(const lego_synth_cfg* c) {
  if (!c) return 0;
  double f = 1.0 + (double)c->dup_frac * 2.0 + 0.01;
  return (int32_t)(c->n_scan * (double)c->horizon_scan * f) + 64;
}

extern "C" int lego_synth_scan(const lego_synth_cfg* c, int32_t k, lego_point_xyzir* out,
                               int32_t cap, int32_t* n_out, double* stamp) {
  if (!c || !out || !n_out || c->n_scan <= 0 || c->horizon_scan <= 0) return LEGO_E_ARG;
  Scene sc = build_scene(*c);
  const int N = c->n_scan, H = c->horizon_scan;
  const double res = 2.0 * M_PI / H;
  const double t0 = (double)k * c->scan_period;
  if (stamp) *stamp = t0;
  std::vector<double> cel(N), sel(N);
  for (int r = 0; r < N; ++r) {
    double el = (c->vert_min_deg + (N > 1 ? (c->vert_max_deg - c->vert_min_deg) * r / (N - 1) : 0.0)) *
                M_PI / 180.0;
    cel[r] = std::cos(el);
    sel[r] = std::sin(el);
  }
  int32_t n = 0;
  const uint64_t skey = c->seed * 0x9E3779B97F4A7C15ULL + (uint64_t)k * 0xD1B54A32D192ED03ULL;
  for (int col = 0; col < H; ++col) {
    double t = t0 + (double)col / H * c->scan_period;
    double px, py, yaw;
    ego_pose(*c, t, &px, &py, &yaw);
    double cy = std::cos(yaw), sy = std::sin(yaw);
    double o[3] = {px, py, 0.0};
    for (int r = 0; r < N; ++r) {
      uint64_t key = skey ^ ((uint64_t)col * 0x632BE59BD9B4E019ULL) ^ ((uint64_t)r * 0x8CB92BA72F3D8DD7ULL);
      double j = (hash_uni(key ^ 0x1111) * 2.0 - 1.0) * c->azimuth_jitter;
      // sensor azimuth sweeps clockwise from just below +pi (image column 0)
      double az = M_PI - (col + 0.25 + j) * res;
      double ds[3] = {cel[r] * std::cos(az), cel[r] * std::sin(az), sel[r]};
      double dw[3] = {cy * ds[0] - sy * ds[1], sy * ds[0] + cy * ds[1], ds[2]};
      double tr = cast(sc, o, dw);
      if (tr > c->max_range) continue;
      if (hash_uni(key ^ 0x2222) < c->dropout) continue;
      int reps = (hash_uni(key ^ 0x3333) < c->dup_frac) ? 2 : 1;
      for (int rep = 0; rep < reps; ++rep) {
        double rr = tr + c->noise_sigma * hash_gauss(key ^ (0x4444 + rep));
        if (rep) rr *= 1.0 + 0.05 * hash_uni(key ^ 0x5555);
        if (n >= cap) return LEGO_E_CAPACITY;
        lego_point_xyzir& p = out[n++];
        std::memset(&p, 0, sizeof(p));
        p.x = (float)(rr * ds[0]);
        p.y = (float)(rr * ds[1]);
        p.z = (float)(rr * ds[2]);
        p.intensity = (float)std::floor(hash_uni(key ^ 0x6666) * 100.0);
        p.ring = (uint16_t)r;
      }
    }
  }
  *n_out = n;
  return LEGO_OK;
}

extern "C" int lego_synth_imu(const lego_synth_cfg* c, double t0, double t1, double rate_hz, double phase,
                              lego_imu_msg* out, int32_t cap, int32_t* n_out) {
  if (!c || !out || !n_out || !(rate_hz > 0) || !(t1 >= t0)) return LEGO_E_ARG;
  const double v = c->speed_mps, w = c->yaw_rate_dps * M_PI / 180.0, g = 9.81;
  const double dt = 1.0 / rate_hz;
  int32_t n = 0;
  for (int64_t i = (int64_t)std::ceil((t0 - phase) * rate_hz - 1e-9);; ++i) {
    const double t = phase + (double)i * dt;
    if (t < t0) continue;
    if (t >= t1) break;
    if (n >= cap) return LEGO_E_CAPACITY;
    // attitude: the ego yaw plus a gentle roll / pitch sway
    const double a1 = 2.0 * M_PI * 0.5, a2 = 2.0 * M_PI * 0.3;
    const double roll = 0.01 * std::sin(a1 * t), pitch = 0.008 * std::sin(a2 * t + 1.0);
    double px, py, yaw;
    ego_pose(*c, t, &px, &py, &yaw);
    const double droll = 0.01 * a1 * std::cos(a1 * t), dpitch = 0.008 * a2 * std::cos(a2 * t + 1.0);
    // quaternion of R = Rz(yaw) Ry(pitch) Rx(roll) (tf setRPY)
    const double hr = roll / 2, hp = pitch / 2, hy = yaw / 2;
    const double cr = std::cos(hr), sr = std::sin(hr), cp = std::cos(hp), sp = std::sin(hp);
    const double cy = std::cos(hy), sy = std::sin(hy);
    lego_imu_msg& m = out[n++];
    std::memset(&m, 0, sizeof(m));
    m.stamp = t;
    m.orientation[0] = sr * cp * cy - cr * sp * sy;
    m.orientation[1] = cr * sp * cy + sr * cp * sy;
    m.orientation[2] = cr * cp * sy - sr * sp * cy;
    m.orientation[3] = cr * cp * cy + sr * sp * sy;
    const uint64_t key = c->seed * 0xA24BAED4963EE407ULL + (uint64_t)i * 0x9FB21C651E98DF25ULL;
    m.angular_velocity[0] = droll + 0.002 * hash_gauss(key ^ 0x71);
    m.angular_velocity[1] = dpitch + 0.002 * hash_gauss(key ^ 0x72);
    m.angular_velocity[2] = w + 0.002 * hash_gauss(key ^ 0x73);
    // specific force: centripetal acceleration plus the gravity reaction, in the body frame
    const double fw[3] = {-v * w * std::sin(yaw), v * w * std::cos(yaw), g};
    const double Cy = std::cos(yaw), Sy = std::sin(yaw), Cp = std::cos(pitch), Sp = std::sin(pitch);
    const double Cr = std::cos(roll), Sr = std::sin(roll);
    // R^T f, R = Rz Ry Rx
    const double a0 = Cy * fw[0] + Sy * fw[1], b0 = -Sy * fw[0] + Cy * fw[1], z0 = fw[2];
    const double a1x = Cp * a0 - Sp * z0, z1 = Sp * a0 + Cp * z0;
    const double fb[3] = {a1x, Cr * b0 + Sr * z1, -Sr * b0 + Cr * z1};
    for (int k = 0; k < 3; ++k) m.linear_acceleration[k] = fb[k] + 0.02 * hash_gauss(key ^ (0x80 + k));
  }
  *n_out = n;
  return LEGO_OK;
}

extern "C" int lego_synth_map(uint64_t seed, float radius, int32_t n_surf, int32_t n_corner,
                              lego_point_xyzi* surf, lego_point_xyzi* corner) {
  if ((n_surf && !surf) || (n_corner && !corner) || radius <= 0) return LEGO_E_ARG;
  Rng r(seed * 0x9E3779B97F4A7C15ULL + 3);
  // Surf: ground plane (camera frame y = -1.2) on a 0.4 m jittered grid, plus
  // building facades (vertical planes); corner: vertical edges (poles) sampled
  // every 0.2 m in height.
  const double h = 1.2;
  int32_t ns = 0;
  int n_ground = n_surf / 2;
  while (ns < n_ground) {
    double x = r.range(-radius, radius), z = r.range(-radius, radius);
    if (x * x + z * z > (double)radius * radius) continue;
    x = std::floor(x / 0.4) * 0.4 + r.range(-0.05, 0.05);
    z = std::floor(z / 0.4) * 0.4 + r.range(-0.05, 0.05);
    surf[ns++] = {(float)x, (float)(-h + r.range(-0.01, 0.01)), (float)z, (float)r.range(0, 100)};
  }
  int n_fac = 24;
  std::vector<double> fx(n_fac), fz(n_fac), fa(n_fac), fl(n_fac);
  for (int i = 0; i < n_fac; ++i) {
    double a = r.range(-M_PI, M_PI), d = r.range(8.0, radius * 0.9);
    fx[i] = d * std::cos(a); fz[i] = d * std::sin(a);
    fa[i] = a + M_PI / 2 + r.range(-0.4, 0.4); fl[i] = r.range(6.0, 20.0);
  }
  while (ns < n_surf) {
    int i = (int)(r.uni() * n_fac) % n_fac;
    double u = std::floor(r.range(-fl[i], fl[i]) / 0.4) * 0.4;
    double y = std::floor(r.range(-h, 8.0) / 0.4) * 0.4;
    double e = r.range(-0.02, 0.02);
    double x = fx[i] + std::cos(fa[i]) * u - std::sin(fa[i]) * e;
    double z = fz[i] + std::sin(fa[i]) * u + std::cos(fa[i]) * e;
    surf[ns++] = {(float)x, (float)y, (float)z, (float)r.range(0, 100)};
  }
  int32_t nc = 0;
  int n_pole = n_corner / 60 + 1;
  std::vector<double> px(n_pole), pz(n_pole);
  for (int i = 0; i < n_pole; ++i) {
    double a = r.range(-M_PI, M_PI), d = r.range(3.0, radius * 0.95);
    px[i] = d * std::cos(a); pz[i] = d * std::sin(a);
  }
  while (nc < n_corner) {
    int i = (int)(r.uni() * n_pole) % n_pole;
    double y = -h + std::floor(r.range(0.0, 12.0) / 0.2) * 0.2;
    corner[nc++] = {(float)(px[i] + r.range(-0.03, 0.03)), (float)y,
                    (float)(pz[i] + r.range(-0.03, 0.03)), (float)r.range(0, 100)};
  }
  return LEGO_OK;
}
