#include "xtc2.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cmath>
#include <cstring>
#include <limits>
#include <algorithm>
#include <map>

#include "common.h"

namespace pr {

int64_t xtc2::type_size(uint32_t t) {
  switch (t) {
    case kUINT8: case kINT8: case kCHARSTR: return 1;
    case kUINT16: case kINT16: return 2;
    case kUINT32: case kINT32: case kFLOAT: return 4;
    case kUINT64: case kINT64: case kDOUBLE: return 8;
    default: return 0;
  }
}

namespace {

using namespace xtc2;

struct XtcHdr {
  uint32_t src;
  uint16_t damage;
  uint16_t contains;
  uint32_t extent;
};
static_assert(sizeof(XtcHdr) == kXtcHeader, "Xtc header is 12 bytes");

struct DgramHdr {
  uint32_t ts_nsec, ts_sec, env;
  XtcHdr xtc;
};
static_assert(sizeof(DgramHdr) == kDgramHeader, "Dgram header is 24 bytes");

struct NameDef {
  std::string name;
  uint32_t type, rank;
};
struct NamesDef {
  std::string det, det_type, alg;
  std::vector<NameDef> names;
};

int64_t pad4(int64_t n) { return (n + 3) & ~int64_t(3); }

// Children of the xtc whose payload spans [p, end): calls f(hdr, payload, payload_end).
template <class F>
void for_children(const uint8_t* p, const uint8_t* end, F&& f) {
  while (p < end) {
    check(end - p >= kXtcHeader, "xtc2: truncated child header");
    XtcHdr h;
    std::memcpy(&h, p, sizeof(h));
    check(h.extent >= (uint32_t)kXtcHeader && (int64_t)h.extent <= end - p, "xtc2: child extent out of bounds");
    f(h, p + kXtcHeader, p + h.extent);
    p += pad4(h.extent);
  }
}

std::string cstr(const uint8_t* p, int n) {
  size_t k = 0;
  while (k < (size_t)n && p[k] != 0) ++k;
  return std::string(reinterpret_cast<const char*>(p), k);
}

NamesDef parse_names(const uint8_t* p, const uint8_t* end) {
  constexpr int kHead = 4 * kNameBytes + 16;
  check(end - p >= kHead, "xtc2: truncated Names");
  NamesDef d;
  d.det = cstr(p, kNameBytes);
  d.det_type = cstr(p + kNameBytes, kNameBytes);
  d.alg = cstr(p + 3 * kNameBytes, kNameBytes);
  uint32_t n;
  std::memcpy(&n, p + 4 * kNameBytes + 8, 4);
  const uint8_t* q = p + kHead;
  check(end - q >= (int64_t)n * (kNameBytes + 8), "xtc2: truncated Name list");
  for (uint32_t i = 0; i < n; ++i, q += kNameBytes + 8) {
    NameDef nd;
    nd.name = cstr(q, kNameBytes);
    std::memcpy(&nd.type, q + kNameBytes, 4);
    std::memcpy(&nd.rank, q + kNameBytes + 4, 4);
    check(type_size(nd.type) > 0 && nd.rank <= (uint32_t)kMaxRank, "xtc2: bad Name type / rank");
    d.names.push_back(nd);
  }
  return d;
}

// One ShapesData: per-variable (shape, data pointer within [data, data_end)).
struct Vars {
  std::vector<std::vector<int64_t>> shape;
  std::vector<int64_t> data_rel;   // offset of each variable from the start of the walked buffer
  std::vector<int64_t> nbytes;
};

// [p, end) is the ShapesData payload; only [p, buf_end) is in memory (buf_end < end when a
// bigdata datagram's head is walked: the Data child's payload -- the raw array -- is not read).
Vars parse_shapes_data(const NamesDef& nd, const uint8_t* base, const uint8_t* p, const uint8_t* end,
                       const uint8_t* buf_end) {
  Vars v;
  const uint8_t* shapes = nullptr;
  const uint8_t* shapes_end = nullptr;
  const uint8_t* data = nullptr;
  const uint8_t* data_end = nullptr;
  while (p < end && (shapes == nullptr || data == nullptr)) {
    check(end - p >= kXtcHeader && buf_end - p >= kXtcHeader, "xtc2: truncated ShapesData child header");
    XtcHdr h;
    std::memcpy(&h, p, sizeof(h));
    check(h.extent >= (uint32_t)kXtcHeader && (int64_t)h.extent <= end - p, "xtc2: child extent out of bounds");
    const uint16_t t = h.contains & 0xff;
    if (t == kShapes) {
      shapes = p + kXtcHeader;
      shapes_end = p + h.extent;
      check(shapes_end <= buf_end, "xtc2: Shapes outside the walked window");
    } else if (t == kData) {
      data = p + kXtcHeader;
      data_end = p + h.extent;
    }
    p += pad4(h.extent);
  }
  check(shapes != nullptr && data != nullptr, "xtc2: ShapesData without Shapes or Data");
  const size_t nv = nd.names.size();
  check(shapes_end - shapes >= (int64_t)(nv * kMaxRank * 4), "xtc2: truncated Shapes");
  int64_t off = 0;
  for (size_t i = 0; i < nv; ++i) {
    uint32_t sh[kMaxRank];
    std::memcpy(sh, shapes + i * kMaxRank * 4, sizeof(sh));
    std::vector<int64_t> s;
    int64_t n = 1;
    for (uint32_t r = 0; r < nd.names[i].rank; ++r) {
      s.push_back(sh[r]);
      n *= sh[r];
    }
    const int64_t nb = n * type_size(nd.names[i].type);
    v.shape.push_back(s);
    v.data_rel.push_back((data - base) + off);
    v.nbytes.push_back(nb);
    off += pad4(nb);
  }
  check(data + off <= data_end, "xtc2: Data shorter than its Shapes say");
  return v;
}

struct Mapped {
  const uint8_t* p = nullptr;
  size_t n = 0;
  explicit Mapped(const std::string& path) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    check(fd >= 0, "xtc2: cannot open " + path);
    struct stat sb;
    check(fstat(fd, &sb) == 0, "xtc2: fstat failed");
    n = (size_t)sb.st_size;
    if (n > 0) {
      void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
      ::close(fd);
      check(m != MAP_FAILED, "xtc2: mmap failed for " + path);
      p = static_cast<const uint8_t*>(m);
    } else {
      ::close(fd);
    }
  }
  ~Mapped() {
    if (p != nullptr) munmap(const_cast<uint8_t*>(p), n);
  }
};

void pread_all(int fd, void* dst, size_t n, off_t off) {
  char* p = static_cast<char*>(dst);
  while (n > 0) {
    const ssize_t r = ::pread(fd, p, n, off);
    if (r < 0 && errno == EINTR) continue;
    check(r > 0, "xtc2: short read of the bigdata file");
    p += r;
    n -= (size_t)r;
    off += r;
  }
}

}  // namespace

Xtc2Index xtc2_scan(const std::string& smd_path, const std::string& big_path, const std::string& det_name,
                    const std::string& array_name) {
  Xtc2Index ix;
  ix.transitions.assign(16, 0);
  std::map<uint32_t, NamesDef> names;
  uint32_t det_id = 0, smd_id = 0, ebeam_id = 0;
  bool have_det = false, have_smd = false, have_ebeam = false;
  int det_var = -1;
  std::vector<int64_t> big_off, big_size;
  const double nan = std::numeric_limits<double>::quiet_NaN();
  {
    Mapped smd(smd_path);
    size_t pos = 0;
    while (pos < smd.n) {
      check(smd.n - pos >= (size_t)kDgramHeader, "xtc2: truncated datagram header in " + smd_path);
      DgramHdr d;
      std::memcpy(&d, smd.p + pos, sizeof(d));
      check(d.xtc.extent >= (uint32_t)kXtcHeader, "xtc2: bad root extent");
      const size_t total = (size_t)(kDgramHeader - kXtcHeader) + d.xtc.extent;
      check(pos + total <= smd.n, "xtc2: datagram runs past the end of " + smd_path);
      const uint32_t service = (d.env >> 24) & 0xf;
      ++ix.transitions[service];
      const uint8_t* body = smd.p + pos + kDgramHeader;
      const uint8_t* body_end = smd.p + pos + total;
      if (service == kConfigure) {
        for_children(body, body_end, [&](const XtcHdr& h, const uint8_t* cp, const uint8_t* ce) {
          if ((h.contains & 0xff) != kNames) return;
          NamesDef nd = parse_names(cp, ce);
          if (nd.det == det_name) {
            for (size_t i = 0; i < nd.names.size(); ++i)
              if (nd.names[i].name == array_name) {
                det_id = h.src;
                det_var = (int)i;
                have_det = true;
                ix.det_type = nd.det_type;
                ix.dtype = nd.names[i].type;
              }
          } else if (nd.det == "smdinfo") {
            smd_id = h.src;
            have_smd = true;
          } else if (nd.det == "ebeam") {
            ebeam_id = h.src;
            have_ebeam = true;
          }
          names[h.src] = std::move(nd);
        });
      } else if (service == kL1Accept) {
        check(have_smd, "xtc2: L1Accept before a Configure with smdinfo Names in " + smd_path);
        int64_t off = -1, size = -1;
        double pe = nan;
        for_children(body, body_end, [&](const XtcHdr& h, const uint8_t* cp, const uint8_t* ce) {
          if ((h.contains & 0xff) != kShapesData) return;
          auto it = names.find(h.src);
          check(it != names.end(), "xtc2: ShapesData with an unknown NamesId");
          const Vars v = parse_shapes_data(it->second, smd.p + pos, cp, ce, ce);
          if (have_smd && h.src == smd_id) {
            check(v.nbytes.size() >= 2 && v.nbytes[0] == 8 && v.nbytes[1] == 8, "xtc2: bad smdinfo record");
            std::memcpy(&off, smd.p + pos + v.data_rel[0], 8);
            std::memcpy(&size, smd.p + pos + v.data_rel[1], 8);
          } else if (have_ebeam && h.src == ebeam_id && !v.nbytes.empty() && v.nbytes[0] == 8) {
            std::memcpy(&pe, smd.p + pos + v.data_rel[0], 8);
          }
        });
        check(off >= 0 && size >= kDgramHeader, "xtc2: L1Accept without an smdinfo offset");
        big_off.push_back(off);
        big_size.push_back(size);
        ix.gevt.push_back((int64_t)ix.gevt.size());
        ix.timestamp.push_back(((int64_t)d.ts_sec << 32) | d.ts_nsec);
        ix.photon_energy.push_back(pe);
      }
      pos += total;
    }
  }
  check(have_det, "xtc2: detector '" + det_name + "' with array '" + array_name + "' not configured in " + smd_path);
  check(!big_off.empty(), "xtc2: no L1Accept in " + smd_path);

  const int fd = ::open(big_path.c_str(), O_RDONLY);
  check(fd >= 0, "xtc2: cannot open " + big_path);
  struct stat sb;
  check(fstat(fd, &sb) == 0, "xtc2: fstat failed");
  const NamesDef& nd = names.at(det_id);
  // walk a bigdata datagram's head (the raw payload itself is not read here)
  std::vector<uint8_t> head(65536);
  auto locate = [&](size_t e) -> int64_t {
    check(big_off[e] + big_size[e] <= (int64_t)sb.st_size, "xtc2: smdinfo points past the end of " + big_path);
    const size_t n = (size_t)std::min<int64_t>((int64_t)head.size(), big_size[e]);
    pread_all(fd, head.data(), n, (off_t)big_off[e]);
    DgramHdr d;
    std::memcpy(&d, head.data(), sizeof(d));
    check(((d.env >> 24) & 0xf) == kL1Accept, "xtc2: smdinfo does not point at an L1Accept");
    check((((int64_t)d.ts_sec << 32) | d.ts_nsec) == ix.timestamp[e], "xtc2: bigdata / smd timestamps differ");
    check((int64_t)(kDgramHeader - kXtcHeader) + d.xtc.extent == big_size[e], "xtc2: datagram size != smdinfo size");
    int64_t rel = -1;
    // the detector's ShapesData comes first in our writer; a head window that cuts a child short
    // is fine as long as the Shapes and the Data header are inside it
    const uint8_t* p = head.data() + kDgramHeader;
    const uint8_t* end = head.data() + big_size[e];
    while (p + kXtcHeader <= head.data() + n && p < end && rel < 0) {
      XtcHdr h;
      std::memcpy(&h, p, sizeof(h));
      check(h.extent >= (uint32_t)kXtcHeader && (int64_t)h.extent <= end - p, "xtc2: child extent out of bounds");
      if ((h.contains & 0xff) == kShapesData && h.src == det_id) {
        const Vars v = parse_shapes_data(nd, head.data(), p + kXtcHeader, p + h.extent, head.data() + n);
        if (ix.shape.empty()) {
          ix.shape = v.shape[det_var];
          ix.frame_bytes = v.nbytes[det_var];
        } else {
          check(v.shape[det_var] == ix.shape, "xtc2: raw array shape changes within the run");
        }
        rel = v.data_rel[det_var];
      }
      p += pad4(h.extent);
    }
    check(rel >= 0, "xtc2: detector data not found in the head of bigdata datagram");
    check(rel + ix.frame_bytes <= big_size[e], "xtc2: raw array runs past its datagram");
    return rel;
  };
  try {
    const int64_t rel0 = locate(0);
    ix.walked = 1;
    const size_t last = big_off.size() - 1;
    if (last > 0 && big_size[last] == big_size[0]) {   // spot-check the same-size assumption
      check(locate(last) == rel0, "xtc2: same-size datagrams with different layouts");
      ++ix.walked;
    }
    ix.payload_off.resize(big_off.size());
    for (size_t e = 0; e < big_off.size(); ++e) {
      // same-size datagrams have the same layout (the writer emits identical ShapesData heads)
      int64_t rel = rel0;
      if (e > 0 && big_size[e] != big_size[0]) {
        rel = locate(e);
        ++ix.walked;
      }
      ix.payload_off[e] = big_off[e] + rel;
    }
  } catch (...) {
    ::close(fd);
    throw;
  }
  ::close(fd);
  check(ix.frame_bytes > 0, "xtc2: empty raw array");
  return ix;
}

}  // namespace pr
