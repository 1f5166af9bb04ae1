// Trajectory ingest: scatter one packed actor record (parallel/trajectory.py pack_rows: header +
// SoA fields at 64-byte aligned offsets) from device memory into an HBM replay sub-ring.
//
// Replaces the reference learner's replay-file ingest (replay_memory.py:155-173 -> :107-119:
// unpickle 233 MB per 5k rows, numpy ring writes) and round 1's host-side ingest_memory (a full
// tree rebuild and a host sync per file).  The record is parsed ON THE DEVICE, so the same
// launch serves records DMA'd from a CPU actor's shared-memory ring (engine/ingest.py) and
// records received over RCCL straight into device memory (RcclTrajectoryChannel.recv_into):
//
//   ingest_rows_kernel  one workgroup per row: frames (16-byte vectors), both stored LSTM states,
//                       the scalars; the sequence-start flag / sum-tree leaf / n_valid follow the
//                       record (the rows it overwrites stop being starts), changed leaves go to
//                       the dirty list (or, for very large records, the caller rebuilds the tree)
//   ingest_tail_kernel  advances the sub-ring's device write head and the rows counter
//
// No host work besides the launch: the write head lives on the device.
//
// Every sub-ring holds ONE producer's stream, written contiguously, so no start outside the
// written rows can go stale: the rows just behind the write head are that stream's newest rows
// (the starts there run on into the rows written now, their true continuation), every row ahead
// of it is untouched old data.  Producers keep each start's window inside the stream they have
// shipped: an actor rank ships overlapping windows (pack_rows_kernel below), a CPU actor whole
// episodes (its last sequence's n-step tail past the episode end is masked by `done`).
#include "../common.h"

#define ING_FIELDS 10   // state hs_cs target_hs_cs action reward done stack_count priority seqprio start
#define ING_MAGIC 0x52324454ll

struct IngestArgs {
  const uint8_t* rec;       // device record
  long long rec_bytes;
  int sub, max_rows;        // destination sub-ring, grid rows (>= rows kept)
  long long* ihead;         // (n_sub) device write heads
  long long* rows_total;    // (1) rows ingested
  unsigned* err;            // bit 0: malformed record
  uint8_t* frames;          // (cap, FB)
  float* hs_cs;             // (cap, 2H)
  float* ths_cs;            // (cap, 2H)
  uint8_t* action;
  float* reward;
  uint8_t* done;
  float* priority;
  uint8_t* is_start;
  float* leaves;
  int* n_valid;
  int* dirty;               // null: no dirty list (the caller rebuilds the tree)
  int* count;
  int max_dirty;
  int FB, H2, cap_e;
  int rows_per_sub;         // > 0: rows i*rps .. (i+1)*rps - 1 go to sub-ring sub + i (an actor
                            // rank's E env blocks in one record); 0: every row to sub-ring sub
  int start_lag;            // rows_per_sub > 0: the start flag / sequence priority of record row j
                            // belong to sub-ring position head + j - start_lag (a start becomes
                            // sampleable with the last row of its window, which arrives start_lag
                            // rows after it); 0: to the row itself
  int n_sub;                // sub-rings of the replay (a record addressing more is rejected)
  int pad_;
};

struct RecView {
  long long n;
  long long off[ING_FIELDS];
  int code[ING_FIELDS];
  long long per_row[ING_FIELDS];
  long long nbytes[ING_FIELDS];
};

__device__ __forceinline__ long long pad64(long long x) { return (x + 63) & ~63ll; }

// false if the record does not match the replay schema
__device__ bool parse_record(const IngestArgs& a, RecView& v) {
  const long long* h = reinterpret_cast<const long long*>(a.rec);
  if (h[0] != ING_MAGIC || h[2] != ING_FIELDS) return false;
  v.n = h[1];
  long long off = pad64(24 + 24 * ING_FIELDS);
  for (int f = 0; f < ING_FIELDS; ++f) {
    v.code[f] = (int)h[3 + 3 * f];
    v.per_row[f] = h[4 + 3 * f];
    v.nbytes[f] = h[5 + 3 * f];
    v.off[f] = off;
    off += pad64(v.nbytes[f]);
  }
  if (off > a.rec_bytes || v.n < 0) return false;
  // every field must hold n rows of its declared width (a header whose n exceeds its payload
  // would make the row scatter read past the record)
  for (int f = 0; f < ING_FIELDS; ++f) {
    if (v.code[f] < 0 || v.code[f] > 2 || v.per_row[f] < 1) return false;
    const long long esz = v.code[f] == 2 ? 4 : 1;
    if (v.nbytes[f] < v.n * v.per_row[f] * esz) return false;
  }
  // state uint8 x FB, states fp32 x 2H, 1-byte or fp32 scalars
  if (v.code[0] != 0 || v.per_row[0] != a.FB) return false;
  if (v.code[1] != 2 || v.per_row[1] != a.H2 || v.code[2] != 2 || v.per_row[2] != a.H2) return false;
  if (v.code[4] != 2 || v.code[7] != 2 || v.code[8] != 2) return false;
  if (v.code[3] == 2 || v.code[9] == 2) return false;
  // env-major blocks: whole blocks only, every addressed sub-ring inside the replay
  if (a.rows_per_sub > 0 &&
      (v.n % a.rows_per_sub != 0 || a.sub + v.n / a.rows_per_sub > a.n_sub)) return false;
  if (a.rows_per_sub <= 0 && a.sub >= a.n_sub) return false;
  return true;
}

__device__ __forceinline__ float scalar_at(const uint8_t* base, int code, long long i) {
  if (code == 2) return reinterpret_cast<const float*>(base)[i];
  if (code == 1) return (float)reinterpret_cast<const int8_t*>(base)[i];
  return (float)base[i];
}

__global__ __launch_bounds__(256) void ingest_rows_kernel(const IngestArgs a) {
  RecView v;
  const bool ok = parse_record(a, v);
  const int tid = threadIdx.x;
  if (!ok) {
    if (blockIdx.x == 0 && tid == 0) atomicOr(a.err, 1u);
    return;
  }
  long long src, row, srow = -1;   // srow: the row whose start flag this block writes
  bool clear_own = true;
  if (a.rows_per_sub > 0) {   // env-major blocks: one per sub-ring, rows_per_sub <= cap_e
    const long long i = blockIdx.x;
    if (i >= v.n) return;
    const int sub = a.sub + (int)(i / a.rows_per_sub);
    const long long j = i % a.rows_per_sub;
    src = i;
    const long long base = (long long)sub * a.cap_e;
    row = base + (a.ihead[sub] + j) % a.cap_e;
    if (a.start_lag > 0) {
      // the record's start column is lagged: it marks position head + j - lag; this row's own
      // start comes with a later block (j + lag < rows_per_sub) or a later record (cleared now)
      srow = base + ((a.ihead[sub] + j - a.start_lag) % a.cap_e + a.cap_e) % a.cap_e;
      clear_own = j + a.start_lag >= a.rows_per_sub;
    }
  } else {
    const long long keep = v.n < a.cap_e ? v.n : a.cap_e;
    const long long i = blockIdx.x;
    if (i >= keep) return;
    src = v.n - keep + i;                                // only the newest cap_e rows survive
    const long long head = a.ihead[a.sub];
    row = (long long)a.sub * a.cap_e + (head + i) % a.cap_e;
  }
  // frames: 16-byte vectors (fields are 64-byte aligned; FB % 16 == 0 for every frame geometry)
  {
    const uint8_t* s = a.rec + v.off[0] + src * a.FB;
    uint8_t* d = a.frames + row * a.FB;
    if ((a.FB & 15) == 0) {
      const int nv = a.FB >> 4;
      for (int k = tid; k < nv; k += blockDim.x)
        reinterpret_cast<u32x4*>(d)[k] = reinterpret_cast<const u32x4*>(s)[k];
    } else {
      for (int k = tid; k < a.FB; k += blockDim.x) d[k] = s[k];
    }
  }
  {
    const float* s1 = reinterpret_cast<const float*>(a.rec + v.off[1]) + src * a.H2;
    const float* s2 = reinterpret_cast<const float*>(a.rec + v.off[2]) + src * a.H2;
    float* d1 = a.hs_cs + row * a.H2;
    float* d2 = a.ths_cs + row * a.H2;
    for (int k = tid; k < a.H2; k += blockDim.x) {
      d1[k] = s1[k];
      d2[k] = s2[k];
    }
  }
  if (tid != 0) return;
  a.action[row] = (uint8_t)(int)scalar_at(a.rec + v.off[3], v.code[3], src);
  a.reward[row] = scalar_at(a.rec + v.off[4], 2, src);
  a.done[row] = scalar_at(a.rec + v.off[5], v.code[5], src) > 0.f ? 1 : 0;
  a.priority[row] = scalar_at(a.rec + v.off[7], 2, src);
  const int st = scalar_at(a.rec + v.off[9], v.code[9], src) != 0.f;
  const float leaf = st ? scalar_at(a.rec + v.off[8], 2, src) : 0.f;
  auto set_start = [&](long long r, int s_, float lf) {
    const int was = a.is_start[r];
    a.is_start[r] = (uint8_t)s_;
    if (was != s_) atomicAdd(a.n_valid, s_ - was);
    if (was || s_ || a.leaves[r] != 0.f) {
      a.leaves[r] = lf;
      if (a.dirty) {
        const int slot = atomicAdd(a.count, 1);
        if (slot < a.max_dirty) a.dirty[slot] = (int)r;
      }
    }
  };
  if (srow < 0) {
    set_start(row, st, leaf);
  } else {
    set_start(srow, st, leaf);
    if (clear_own) set_start(row, 0, 0.f);
  }
}

__global__ void ingest_tail_kernel(const IngestArgs a) {
  if (threadIdx.x != 0) return;
  // the head and the counter advance only for a record the rows kernel accepted (same parse)
  RecView v;
  if (!parse_record(a, v)) return;
  if (a.rows_per_sub > 0) {
    const int nsub = (int)(v.n / a.rows_per_sub);
    for (int q = 0; q < nsub; ++q) a.ihead[a.sub + q] = (a.ihead[a.sub + q] + a.rows_per_sub) % a.cap_e;
    *a.rows_total += v.n;
    return;
  }
  const long long keep = v.n < a.cap_e ? v.n : a.cap_e;
  a.ihead[a.sub] = (a.ihead[a.sub] + keep) % a.cap_e;
  *a.rows_total += keep;
}

extern "C" int r2_ingest_args_bytes() { return (int)sizeof(IngestArgs); }

// ---------------------------------------------------------------------------------------------
// The producer side of a device record: an actor rank's replay rows [h0, h0 + K) of each of its E
// sub-rings (ring-wrapped), env-major, into a record whose header the caller wrote once (fixed
// E, K: a constant layout).  Only the starts whose whole window lies inside the record are kept
// (start_from <= j < start_to): consecutive windows overlap by W - 1 rows, so every sequence is
// shipped exactly once and the learner never samples a window it has not fully received.  Replaces the host-side pack_rows of the RCCL trajectory channel:
// the rows never leave device memory on either side of the send.
struct PackArgs {
  const uint8_t* frames; const float* hs_cs; const float* ths_cs; const uint8_t* action;
  const float* reward; const uint8_t* done; const float* priority; const uint8_t* is_start;
  const float* leaves;
  uint8_t* rec;
  long long off[ING_FIELDS];   // byte offset of every field in the record
  long long h0;                // first ring position (same for every sub-ring: lockstep envs)
  int E, K, cap_e, FB, H2;     // K rows per env block
  int start_from, start_to;    // starts kept only for block rows j in [start_from, start_to)
  int lag;                     // the start column of row j describes ring position h0 + j - lag
};

__global__ __launch_bounds__(256) void pack_rows_kernel(const PackArgs a) {
  const int i = blockIdx.x;                // record row (env-major)
  const int e = i / a.K, j = i % a.K;
  const long long row = (long long)e * a.cap_e + (a.h0 + j) % a.cap_e;
  const int tid = threadIdx.x;
  {
    const u32x4* s = reinterpret_cast<const u32x4*>(a.frames + row * a.FB);
    u32x4* d = reinterpret_cast<u32x4*>(a.rec + a.off[0] + (long long)i * a.FB);
    for (int k = tid; k < a.FB / 16; k += blockDim.x) d[k] = s[k];
  }
  {
    float* d1 = reinterpret_cast<float*>(a.rec + a.off[1]) + (long long)i * a.H2;
    float* d2 = reinterpret_cast<float*>(a.rec + a.off[2]) + (long long)i * a.H2;
    for (int k = tid; k < a.H2; k += blockDim.x) {
      d1[k] = a.hs_cs[row * a.H2 + k];
      d2[k] = a.ths_cs[row * a.H2 + k];
    }
  }
  if (tid != 0) return;
  a.rec[a.off[3] + i] = a.action[row];                                // int8 (A <= 127)
  reinterpret_cast<float*>(a.rec + a.off[4])[i] = a.reward[row];
  reinterpret_cast<float*>(a.rec + a.off[5])[i] = a.done[row] ? 1.f : 0.f;
  a.rec[a.off[6] + i] = 0;                                           // stack_count
  reinterpret_cast<float*>(a.rec + a.off[7])[i] = a.priority[row];
  const long long srow = (long long)e * a.cap_e + ((a.h0 + j - a.lag) % a.cap_e + a.cap_e) % a.cap_e;
  const bool st = a.is_start[srow] && j >= a.start_from && j < a.start_to;
  reinterpret_cast<float*>(a.rec + a.off[8])[i] = st ? a.leaves[srow] : 0.f;
  a.rec[a.off[9] + i] = st ? 1 : 0;
}

extern "C" int r2_pack_args_bytes() { return (int)sizeof(PackArgs); }

extern "C" int r2_pack_rows(const PackArgs* a, void* stream) {
  if (!a->rec || a->E <= 0 || a->K <= 0 || a->K > a->cap_e || (a->FB & 15) || a->H2 <= 0) return -1;
  if ((reinterpret_cast<uintptr_t>(a->rec) & 63) != 0) return -2;
  hipLaunchKernelGGL(pack_rows_kernel, dim3(a->E * a->K), dim3(256), 0, (hipStream_t)stream, *a);
  R2_CHECK_LAUNCH();
  return 0;
}

// One record -> one sub-ring.  max_rows bounds the grid (rows kept = min(n, cap_e) <= max_rows is
// the caller's contract: it knows the record length, and rows / record >= FB bytes each).
extern "C" int r2_ingest_record(const IngestArgs* a, void* stream) {
  if (!a->rec || a->max_rows <= 0 || a->cap_e <= 0 || a->FB <= 0 || a->H2 <= 0) return -1;
  if ((reinterpret_cast<uintptr_t>(a->rec) & 63) != 0) return -2;
  const int rps = a->rows_per_sub;
  if (rps > a->cap_e) return -3;
  const int grid = rps > 0 ? a->max_rows : (a->max_rows < a->cap_e ? a->max_rows : a->cap_e);
  hipLaunchKernelGGL(ingest_rows_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, *a);
  hipLaunchKernelGGL(ingest_tail_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, *a);
  R2_CHECK_LAUNCH();
  return 0;
}
