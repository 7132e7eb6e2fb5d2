// lego_wire.hip — the ROS wire formats around the hot path (SURVEY.md §8f
// rank 2).
//
//   k_pc2_decode   1 lane / point: pcl::fromROSMsg of a sensor_msgs/PointCloud2
//                  into PointXYZIR (imageProjection.cpp:166, 172) for a batch
//                  of messages in one launch.  A byte gather: HBM-bound, 2 x
//                  point_step-ish bytes per point.
//   host           the PCL field mapping (name + datatype + count), the
//                  PointXYZI encoder (pcl::toROSMsg) and the ROS1 serialiser of
//                  cloud_msgs/cloud_info.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

#include "lego_loam.h"
#include "lego_wire.h"

namespace lego {

// PointXYZIR (utility.h:153-165): x, y, z, intensity FLOAT32, ring UINT16.
static const struct {
  const char* name;
  uint8_t datatype;
  int structOffset, size;
} kXyzirFields[kPc2Fields] = {{"x", LEGO_PF_FLOAT32, 0, 4},
                              {"y", LEGO_PF_FLOAT32, 4, 4},
                              {"z", LEGO_PF_FLOAT32, 8, 4},
                              {"intensity", LEGO_PF_FLOAT32, 16, 4},
                              {"ring", LEGO_PF_UINT16, 20, 2}};

// pcl::detail::FieldMatches + createMapping: a struct field is filled from
// the message field of the same name, datatype and count (1, or 0 for
// scalars); otherwise it is skipped and stays at its value-initialised 0.
int pc2_plan(const lego_pc2_msg* m, Pc2Desc* d) {
  if (!m || m->is_bigendian || m->point_step == 0 || m->n_fields < 0 || (m->n_fields > 0 && !m->fields))
    return LEGO_E_ARG;
  if (m->width > 0 && m->height > 0 && (uint64_t)m->row_step < (uint64_t)m->width * m->point_step)
    return LEGO_E_ARG;
  std::memset(d, 0, sizeof(*d));
  d->data = m->data;
  d->height = m->height;
  d->width = m->width;
  d->pointStep = m->point_step;
  d->rowStep = m->row_step;
  for (int f = 0; f < kPc2Fields; ++f) {
    d->off[f] = -1;
    for (int i = 0; i < m->n_fields; ++i) {
      const lego_pc2_field& mf = m->fields[i];
      if (std::strncmp(mf.name, kXyzirFields[f].name, sizeof(mf.name)) != 0) continue;
      if (mf.datatype != kXyzirFields[f].datatype) continue;
      if (mf.count != 1 && mf.count != 0) continue;
      if (mf.offset + (uint32_t)kXyzirFields[f].size > m->point_step) return LEGO_E_ARG;
      d->off[f] = (int)mf.offset;
      break;
    }
  }
  return LEGO_OK;
}

__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__global__ void k_pc2_decode(const Pc2Desc* descs, lego_point_xyzir* out) {
  const Pc2Desc& d = descs[blockIdx.y];
  const uint64_t n = (uint64_t)d.height * d.width;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t row = i / d.width, col = i - row * d.width;
  const uint8_t* src = d.data + row * d.rowStep + col * d.pointStep;
  uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int f = 0; f < 4; ++f)
    if (d.off[f] >= 0) w[f < 3 ? f : 4] = ld_u32(src + d.off[f]);  // x y z @0-11, intensity @16
  if (d.off[4] >= 0) w[5] = (uint32_t)src[d.off[4]] | ((uint32_t)src[d.off[4] + 1] << 8);
  uint4* o = reinterpret_cast<uint4*>(out + d.outBase + i);
  o[0] = make_uint4(w[0], w[1], w[2], w[3]);
  o[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

int launch_pc2_decode(const Pc2Desc* dDescs, int K, uint64_t maxPoints, lego_point_xyzir* out, hipStream_t s) {
  if (K <= 0 || maxPoints == 0) return 0;
  const dim3 grid((unsigned)((maxPoints + 255) / 256), (unsigned)K);
  k_pc2_decode<<<grid, 256, 0, s>>>(dDescs, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace lego

using namespace lego;

extern "C" int lego_pc2_encode_xyzi(const lego_point_xyzi* pts, int32_t n, uint8_t* data,
                                    lego_pc2_field* fields4) {
  if (n < 0 || (n > 0 && (!pts || !data))) return LEGO_E_ARG;
  // pcl::PointXYZI: x y z data[3] (= 1.0f from its constructor), intensity, 3 pad floats
  const float one = 1.0f;
  for (int32_t i = 0; i < n; ++i) {
    uint8_t* p = data + (size_t)i * 32;
    std::memset(p, 0, 32);
    std::memcpy(p, &pts[i].x, 12);
    std::memcpy(p + 12, &one, 4);
    std::memcpy(p + 16, &pts[i].intensity, 4);
  }
  if (fields4) {
    const char* names[4] = {"x", "y", "z", "intensity"};
    const uint32_t offs[4] = {0, 4, 8, 16};
    for (int f = 0; f < 4; ++f) {
      std::memset(&fields4[f], 0, sizeof(fields4[f]));
      std::strncpy(fields4[f].name, names[f], sizeof(fields4[f].name) - 1);
      fields4[f].offset = offs[f];
      fields4[f].datatype = LEGO_PF_FLOAT32;
      fields4[f].count = 1;
    }
  }
  return LEGO_OK;
}

namespace {
struct Writer {
  uint8_t* buf;
  uint64_t cap, len = 0;
  bool ok = true;
  void put(const void* p, uint64_t n) {
    if (buf) {
      if (len + n > cap) ok = false;
      else std::memcpy(buf + len, p, n);
    }
    len += n;
  }
  void u32(uint32_t v) { put(&v, 4); }  // ROS1 serialisation is little-endian
  void arr(const void* p, uint32_t n, uint32_t esz) {
    u32(n);
    if (n) put(p, (uint64_t)n * esz);
  }
};
}  // namespace

extern "C" int lego_cloud_info_serialize(const lego_cloud_info* info, int32_t n_scan, int32_t horizon_scan,
                                         uint32_t seq, const char* frame_id, uint8_t* buf, uint64_t cap,
                                         uint64_t* len) {
  if (!info || !len || n_scan <= 0 || horizon_scan <= 0) return LEGO_E_ARG;
  const uint32_t N = (uint32_t)n_scan, P = (uint32_t)n_scan * (uint32_t)horizon_scan;
  if (!info->start_ring_index || !info->end_ring_index || !info->segmented_cloud_ground_flag ||
      !info->segmented_cloud_col_ind || !info->segmented_cloud_range)
    return LEGO_E_ARG;
  // ros::Time::fromSec (rostime/impl/time.h): sec = floor(t), nsec = round((t - sec) * 1e9)
  const double t = info->stamp;
  if (!(t >= 0) || t > 4294967295.0) return LEGO_E_ARG;
  uint32_t sec = (uint32_t)std::floor(t);
  uint64_t nsec = (uint64_t)std::llround((t - sec) * 1e9);
  if (nsec >= 1000000000ull) { sec += (uint32_t)(nsec / 1000000000ull); nsec %= 1000000000ull; }
  Writer w{buf, cap};
  w.u32(seq);
  w.u32(sec);
  w.u32((uint32_t)nsec);
  const char* fid = frame_id ? frame_id : "";
  w.arr(fid, (uint32_t)std::strlen(fid), 1);
  w.arr(info->start_ring_index, N, 4);
  w.arr(info->end_ring_index, N, 4);
  w.put(&info->start_orientation, 4);
  w.put(&info->end_orientation, 4);
  w.put(&info->orientation_diff, 4);
  w.arr(info->segmented_cloud_ground_flag, P, 1);  // bool[]: one byte each
  w.arr(info->segmented_cloud_col_ind, P, 4);
  w.arr(info->segmented_cloud_range, P, 4);
  *len = w.len;
  return (buf && !w.ok) ? LEGO_E_CAPACITY : LEGO_OK;
}
