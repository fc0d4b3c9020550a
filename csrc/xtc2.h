// XTC2-style run files: native scanner of the small-data (smd) file + bigdata payload locator.
//
// Reference parity: the reference's events come from psana's XTC2 reader in small-data mode --
// `PsanaWrapperSmd(exp, run, detector_name).iter_events(mode)` (psana_ray/producer.py:11,88,150-154;
// SURVEY E-01, P-01).  psana's SMD mode walks a small per-stream index file whose L1Accept
// datagrams carry the offset/size of the matching datagram in the big data file, and hands MPI
// ranks batches of events to read.  Here the same two-file layout is scanned ONCE in C++; the result
// is a per-event table (payload offset of the detector's raw array in the bigdata file, event id,
// timestamp, photon energy) that RawRunReader's thread pool uses to pread frames straight into
// pinned staging pages (no per-event Python, no copy of the datagram headers).
//
// Container layout (little endian; structure follows LCLS-II xtcdata, byte-exactness with psana
// is NOT pinned -- there is no psana or XTC2 fixture offline):
//   Dgram  = u32 ts_nsec, u32 ts_sec, u32 env (TransitionId in bits 24..27), Xtc root (Parent)
//   Xtc    = u32 src (NamesId = node << 8 | index), u16 damage, u16 contains (version << 8 | type),
//            u32 extent (header included; payloads padded to 4 bytes)
//   Names  (Configure): char detName[256], detType[256], detId[256], algName[256], u32 algVersion,
//            u32 segment, u32 nNames, u32 reserved, then nNames x {char name[256], u32 type, u32 rank}
//   ShapesData (L1Accept, src = the NamesId of its Names): Shapes child (u32[5] per Name) then a
//            Data child (each variable in Name order, padded to 4 bytes)
//   smd L1Accept: ShapesData of det "smdinfo" {u64 intOffset, u64 intDgramSize} (+ "ebeam")
//   bigdata L1Accept: ShapesData of the detector (raw array) + "ebeam" {f64 ebeamPhotonEnergy}
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

namespace pr {

namespace xtc2 {
enum Transition : uint32_t {
  kClearReadout = 0, kReset = 1, kConfigure = 2, kUnconfigure = 3, kBeginRun = 4, kEndRun = 5,
  kBeginStep = 6, kEndStep = 7, kEnable = 8, kDisable = 9, kSlowUpdate = 10, kL1Accept = 12,
};
enum Type : uint16_t { kParent = 0, kShapesData = 1, kShapes = 2, kData = 3, kNames = 4 };
enum DataType : uint32_t {
  kUINT8 = 0, kUINT16, kUINT32, kUINT64, kINT8, kINT16, kINT32, kINT64, kFLOAT, kDOUBLE, kCHARSTR,
};
constexpr int kMaxRank = 5;
constexpr int kNameBytes = 256;
constexpr int kDgramHeader = 24;
constexpr int kXtcHeader = 12;
int64_t type_size(uint32_t t);
}  // namespace xtc2

struct Xtc2Index {
  std::string det_type;
  std::vector<int64_t> shape;        // the raw array's shape (from the first L1Accept)
  uint32_t dtype = 0;                // xtc2::DataType of the raw array
  int64_t frame_bytes = 0;
  std::vector<int64_t> payload_off;  // per L1Accept: byte offset of the raw array in the bigdata file
  std::vector<int64_t> gevt;         // per L1Accept: event counter in the run
  std::vector<int64_t> timestamp;    // per L1Accept: ts_sec << 32 | ts_nsec
  std::vector<double> photon_energy; // per L1Accept: NaN when the event has no ebeam record
  std::vector<int64_t> transitions;  // count per TransitionId (16 entries) in the smd file
  int64_t walked = 0;                // bigdata datagrams whose headers were walked (size changed)
};

// Scans `smd_path`, locates `array_name` of detector `det_name` inside the bigdata file `big_path`.
Xtc2Index xtc2_scan(const std::string& smd_path, const std::string& big_path, const std::string& det_name,
                    const std::string& array_name);

}  // namespace pr
