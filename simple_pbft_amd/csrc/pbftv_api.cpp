// pbftv_api.cpp -- the C ABI of include/pbftv.h on top of the gfx950 kernels.
//
// One pbftv_ctx owns, per GPU: a non-blocking HIP stream, the comb tables of
// G and every registered key (resident in HBM; see choose_bits), and
// grow-only scratch.  Host-buffer batches are cut into contiguous shards
// (multiples of 512 items, so every shard's bitmap starts on a byte and every
// wave on a 64-item boundary), one per device, each driven by its own host
// thread; the shards are independent and the bitmaps are concatenated -- no
// collective.  There is no CPU path: if no gfx950 device is
// usable, pbftv_open fails with PBFTV_ENODEV.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <initializer_list>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pbftv.h"
#include "gojson.h"
#include "gojson_enc.h"
#include "kernels.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

// inside helpers returning hipError_t
#define HIP_TRY_E(expr)             \
  do {                              \
    hipError_t e2_ = (expr);        \
    if (e2_ != hipSuccess) return e2_; \
  } while (0)

#define HIP_TRY(expr)                                                                                         \
  do {                                                                                                        \
    hipError_t e_ = (expr);                                                                                   \
    if (e_ != hipSuccess)                                                                                     \
      return fail(e_ == hipErrorOutOfMemory ? PBFTV_ENOMEM : PBFTV_EDEVICE,                                   \
                  std::string(#expr) + ": " + hipGetErrorString(e_));                                         \
  } while (0)

// ---- armed latency kernels, process-wide (k_ecdsa_wave_armed) ----
// An armed kernel stays resident on its GPU between latency-path calls, and
// hipFree / hipHostFree / hipDeviceSynchronize wait for every kernel on the
// GPU.  So every library path that frees memory or synchronises a whole device
// first QUIESCES that GPU: it bumps the `halt` word of every registered mailbox
// on it (each armed kernel was launched with the value it then held and leaves
// within one poll of a change, reporting `expired`, which sends its owner's
// next call through a launch), and no context arms a kernel on that GPU until
// the quiesce ends.  Other contexts' kernels are cancelled without their locks:
// the mailbox words are host memory and the halt bump is one atomic add.
struct ArmRegistry {
  std::mutex mu;
  std::map<int, std::vector<pbftv::QcMail*>> mail;              // GPU -> registered mailboxes
  std::map<int, std::vector<std::condition_variable*>> keepers;  // GPU -> their devices' keeper wake-ups
  std::map<int, int> quiesce;                                   // GPU -> quiesces in progress
  // The armed kernels' streams take high-priority hardware queues, and the
  // runtime keeps only GPU_MAX_HW_QUEUES (4) of them per GPU: a fifth stream
  // shares one, and a kernel launched there waits for the resident kernel's
  // whole budget (tools/hiq_share.hip, profiles/r06_hiq_share.txt).  So the
  // contexts of a process hold at most that many between them, a pair each
  // (qc_streams_ready); a context without one launches its certificates on a
  // normal-priority stream until a holder that has been idle gives its pair up.
  std::map<int, int> hiq_pairs;                                           // GPU -> pairs held
  std::map<int, std::chrono::steady_clock::time_point> hiq_wanted;       // GPU -> a context last found none free
};
ArmRegistry& arm_registry() {
  static ArmRegistry* r = new ArmRegistry;  // never destroyed: DevBuf destructors may run at exit
  return *r;
}

// gpu < 0: every GPU (a pinned host buffer is not tied to one device)
void halt_armed_locked(ArmRegistry& r, int gpu) {
  for (auto& kv : r.mail)
    if (gpu < 0 || kv.first == gpu)
      for (pbftv::QcMail* m : kv.second) __atomic_add_fetch(&m->halt, 1u, __ATOMIC_RELEASE);
}

bool arming_allowed_locked(ArmRegistry& r, int gpu) { return r.quiesce[gpu] == 0 && r.quiesce[-1] == 0; }

struct GpuQuiesce {
  int gpu;  // < 0: all
  explicit GpuQuiesce(int g) : gpu(g) {
    ArmRegistry& r = arm_registry();
    std::lock_guard<std::mutex> lk(r.mu);
    ++r.quiesce[gpu];
    halt_armed_locked(r, gpu);
  }
  ~GpuQuiesce() {
    ArmRegistry& r = arm_registry();
    std::lock_guard<std::mutex> lk(r.mu);
    --r.quiesce[gpu];
    // the halted servers' keepers re-arm now, not at their next half budget
    // (a certificate in between would take a launch)
    for (auto& kv : r.keepers)
      if ((gpu < 0 || kv.first == gpu) && arming_allowed_locked(r, kv.first))
        for (std::condition_variable* cv : kv.second) cv->notify_one();
  }
  GpuQuiesce(const GpuQuiesce&) = delete;
  GpuQuiesce& operator=(const GpuQuiesce&) = delete;
};

int current_gpu() {
  int g = 0;
  (void)hipGetDevice(&g);
  return g;
}

// grow-only device buffer (a free quiesces the current GPU first)
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  unsigned flags = 0;  // hipExtMallocWithFlags flags (0: plain hipMalloc)
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) {
      GpuQuiesce q(current_gpu());
      (void)hipFree(p);
    }
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 4096);
    hipError_t e = flags ? hipExtMallocWithFlags(&p, want, flags) : hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) {
      GpuQuiesce q(current_gpu());
      (void)hipFree(p);
    }
    p = nullptr;
    cap = 0;
  }
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

// pinned, device-coherent host memory: kernels read inputs from and write
// results to it directly (the small-batch latency path: no DMA copies)
struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  unsigned flags = hipHostMallocCoherent | hipHostMallocMapped;  // plain pinned (DMA staging): hipHostMallocDefault
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) {
      GpuQuiesce q(-1);
      (void)hipHostFree(p);
    }
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 1 << 16);
    hipError_t e = hipHostMalloc(&p, want, flags);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) {
      GpuQuiesce q(-1);
      (void)hipHostFree(p);
    }
    p = nullptr;
    cap = 0;
  }
  HostBuf() = default;
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  ~HostBuf() { release(); }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

// Device scratch of one lane-path verify (stage-1 records, prefix products of
// the batched inversion, key order, per-signature result bytes).
struct VerifyScratch {
  DevBuf rec, prefix, ksort, okb;
  uint32_t sort_parity = 0;  // batches sorted with ksort (launch_key_count's counter sets)
  void release() {
    rec.release();
    prefix.release();
    ksort.release();
    okb.release();
  }
};

struct Device {
  int id = -1;
  hipStream_t stream = nullptr;
  std::mutex mu;
  // ---- what a latency-path call reads and writes, together from here to
  // hot_end (prefetched at its entry: a certificate after an idle second finds
  // them cold, and one line per miss would serialise behind the lock) ----
  bool have_keys = false;
  bool mail_registered = false;  // the mailbox is in the arm registry
  bool keeper_stop = false, keeper_idle = false;
  bool qc_armed_served = false;
  HostBuf stage;  // zero-copy inputs/outputs of the small-batch path (a QcMail mailbox)
  // the armed latency kernel (k_ecdsa_wave_armed): a persistent server that
  // waits for the next request's doorbell in `stage`; arm_seq = the request
  // number it waits for (0: none armed)
  // (arm_seq is written under d.mu; latency_device reads other devices' without their locks)
  std::atomic<uint32_t> arm_seq{0};
  uint32_t seq_counter = 0;                // (the armed kernel serves arm_seq, arm_seq + 1, ...)
  int arm_stream = 1;                      // qstream index of the armed kernel
  uint32_t armed_first = 0;                // the armed kernel's first number (its `live` report)
  uint32_t retiring = 0;                   // a rotated-out kernel still waiting for arm_seq's to start
  uint32_t arm_waves = 0;                  // signatures the armed kernel serves: its slots (narrow) or workgroups (wide)
  bool arm_wide = false;                   // the armed kernel is the wide one (helpers fed by the relay)
  uint32_t qc_nmax = 0;                    // largest narrow certificate since the last arming
  uint32_t qc_nmax_prev = 0;               // ... and in the period before (slots shrink only after two)
  uint32_t qc_slots = 4;                   // slots the next narrow arming takes (the row schedule: a CU each)
  uint32_t qc_wmax = 0;                    // largest wide certificate (9..kQcCap) since the last arming
  uint32_t qc_wslots = 0;                  // workgroups of the wide arming (grows while wide is wanted; 0: none yet)
  bool arm_live = false;                   // every workgroup of the armed kernel has reported itself resident
  std::chrono::steady_clock::time_point last_wide{};  // the last latency-path call of 9..kQcCap signatures
  std::chrono::steady_clock::time_point armed_at{}, last_qc{};
  // diagnostics of the last latency-path call (pbftv_qc_stamps)
  uint64_t qc_ns_entry = 0, qc_ns_handover = 0, qc_ns_total = 0, qc_ns_slots = 0;
  char hot_end[1] = {};
  // counters of the latency path since the context opened (pbftv_qc_counters)
  uint64_t qc_calls = 0, qc_armed = 0, qc_reruns = 0, qc_exact_sigs = 0, qc_launches = 0, qc_armings = 0;
  // when the lane-path batches enqueued so far are expected to finish
  // (steady-clock ns; an estimate from their sizes, kept without a HIP call):
  // a multi-device context sends a certificate to its least-loaded device
  std::atomic<int64_t> busy_until_ns{0};
  // signature state: comb table of G (width gbits) and one table per registered
  // key (width qbits), addressed through qptrs (device array, by key).  Key
  // tables live in blocks (one per registration / add_keys call; slots beyond
  // nkeys are spare capacity kept for the next registration at this width).
  std::shared_ptr<DevBuf> gtab;  // shared by every context on this GPU at this width (g_tables)
  DevBuf key_valid, qptrs;
  DevBuf tab_scratch[6];  // table build: bases, L, H, phase-2 / phase-3 scratch, table addresses
  DevBuf tab_keys;        // table build: the keys' coordinates
  std::vector<std::unique_ptr<DevBuf>> qblocks;
  std::vector<void*> qtab;  // table of key j (registered keys first, then spare slots)
  int gbits = 0, qbits = 0;
  uint32_t nkeys = 0;
  // ecdsa scratch
  DevBuf hashes, sigs, key_idx, bitmap;
  VerifyScratch vs;  // the lane path's stage-1 records, prefix products, key order, result bytes
  // the armed kernels' streams, relay words and keeper thread
  hipStream_t qstream[2] = {nullptr, nullptr};  // alternate armings: a rotation's successor spins beside its predecessor
  std::chrono::steady_clock::time_point qstream_given_up{};  // when this context last gave its pair to another (qc_streams_release)
  hipStream_t lstream = nullptr;  // launched latency-path kernels: never queued behind a batch on d.stream
  DevBuf cuflag;                           // certificate flags per CU (kCuFlagWords; zeroed at the first arming)
  std::atomic<uint32_t*> cuflag_ready{nullptr};  // cuflag once zeroed (read by batch launches without the lock)
  DevBuf qrelay;                           // the wide kernels' relay words, one 64-B line per qstream:
                                           // uncached device memory (read and written past the 8 XCDs' L2s, so
                                           // no cache maintenance: an agent-scope acquire per poll would
                                           // invalidate the poller's whole L2)
  std::thread keeper;  // qc_keeper_loop
  std::condition_variable keeper_cv;
  uint64_t rotations = 0;
  // host-buffer pipeline (pbftv_ecdsa_p256_verify_batch above the latency
  // path): two slots of pinned staging + device inputs, a copy stream
  static constexpr int kSlots = 16;  // chunks staged ahead at most (PBFTV_HOST_SLOTS, default 16)
  hipStream_t cstream = nullptr;     // the copies, in chunk order (one DMA queue keeps the link busy)
  hipStream_t stream2 = nullptr;     // the odd chunks' verifies (their own scratch vs2), so two chunks can overlap
  VerifyScratch vs2;
  hipEvent_t join_ev = nullptr;
  DevBuf din[kSlots], keys_all;
  hipEvent_t h2d_ev[kSlots] = {}, comp_ev[kSlots] = {};
  // sha scratch
  DevBuf data, offsets, lengths, order, order_scratch, digests, expected, shabits;
  // message batches (Go-JSON on the device): packed column inputs, verifyMsg bytes,
  // pinned staging for the one H2D and the results
  DevBuf arena, msgok;
  HostBuf mstage, mout;
  HostBuf sstage;  // zero-copy inputs/digests of small digest calls (sha_host_small)
  // pbftv_dev_alloc / pbftv_dev_free: a stream-ordered pool of the library's
  // own, so a caller's free neither synchronises the GPU nor halts the armed
  // servers.  A freed block waits in pending_frees until every stream of the
  // context has passed the point where the free was called (events polled on
  // the host, no stream waits on the GPU), then returns to the pool
  struct PendingFree {
    void* p;
    std::vector<hipEvent_t> ev;
  };
  hipMemPool_t pool = nullptr;
  hipStream_t astream = nullptr;
  std::set<void*> pool_ptrs;
  std::vector<PendingFree> pending_frees;
  std::vector<hipEvent_t> spare_ev;
  // Device scratch (rec, prefix, ksort, okb, order_scratch) is shared by
  // calls on d.stream and on caller streams (the *_dev entry points).  The
  // mutex orders the enqueues; this event orders the execution: a call on a
  // different stream than the last scratch user first waits for it.
  hipEvent_t scratch_ev = nullptr;
  hipStream_t scratch_st = nullptr;
  bool scratch_lazy = false;  // scratch_st == stream: scratch_ev not yet recorded for its last use
  // streams made by pbftv_stream_create own their verify scratch: ECDSA
  // verifies on two such streams run concurrently (batch j + 1's scalar stage
  // in the wave slots batch j's comb leaves free) instead of queueing on d.vs
  std::map<hipStream_t, std::unique_ptr<VerifyScratch>> stream_scratch;
  // caller streams the library did not create that a wave-path verify (no
  // device scratch, so no scratch_ev fence) was enqueued on since the last key
  // change: an event recorded after each such enqueue (events stay valid when
  // the caller destroys its stream); ctx_quiesce waits for them all
  std::map<hipStream_t, hipEvent_t> reader_ev;
  // kernel timing (events recorded around launches while ctx timing is on)
  const bool* timing = nullptr;
  const std::atomic<uint64_t>* wave_max = nullptr;  // the context's latency-path threshold
  static constexpr int kKernels = 5;  // PBFTV_K_*
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending[kKernels];
  double acc_ms[kKernels] = {0, 0, 0, 0, 0};
  uint64_t launches[kKernels] = {0, 0, 0, 0, 0};
};

// key-order scratch: a fresh allocation gets its header zeroed (the sort's
// kernels leave it zero after every batch; p256_kernels.hip k_key_hist).
// st == nullptr: a blocking memset.
hipError_t ensure_key_sort(VerifyScratch& sc, uint64_t n, uint32_t nkeys, hipStream_t st) {
  const size_t cap0 = sc.ksort.cap;
  hipError_t e = sc.ksort.ensure(pbftv::key_sort_scratch_bytes(n, nkeys));
  if (e != hipSuccess || sc.ksort.cap == cap0) return e;
  return st ? hipMemsetAsync(sc.ksort.p, 0, pbftv::key_sort_header_bytes(), st)
            : hipMemset(sc.ksort.p, 0, pbftv::key_sort_header_bytes());
}

// before / after enqueueing work that uses the device scratch on stream st.
// A caller stream's use is fenced by an event recorded right after it.  The
// library's own stream (d.stream, which lives as long as the context) is fenced
// lazily: its event is recorded only when another stream next wants the
// scratch -- recording later on the same stream covers at least the scratch
// work -- so back-to-back calls on d.stream queue no marker between batches
// (each marker costs the GPU a ~6 us gap between kernels, rocprof timeline).
hipError_t scratch_acquire(Device& d, hipStream_t st) {
  if (d.scratch_st == nullptr || d.scratch_st == st) return hipSuccess;
  if (d.scratch_lazy) {
    if (!d.scratch_ev) {
      hipError_t e = hipEventCreateWithFlags(&d.scratch_ev, hipEventDisableTiming);
      if (e != hipSuccess) return e;
    }
    hipError_t e = hipEventRecord(d.scratch_ev, d.scratch_st);
    if (e != hipSuccess) return e;
    d.scratch_lazy = false;
  }
  return hipStreamWaitEvent(st, d.scratch_ev, 0);
}

hipError_t scratch_release(Device& d, hipStream_t st) {
  d.scratch_st = st;
  d.scratch_lazy = st == d.stream;
  if (d.scratch_lazy) return hipSuccess;
  if (!d.scratch_ev) {
    hipError_t e = hipEventCreateWithFlags(&d.scratch_ev, hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  return hipEventRecord(d.scratch_ev, st);
}

// record start/stop events around one launch when timing is enabled
template <class F>
hipError_t timed(Device& d, int k, hipStream_t st, F launch) {
  if (!d.timing || !*d.timing) return launch();
  hipEvent_t a, b;
  hipError_t e = hipEventCreate(&a);
  if (e != hipSuccess) return e;
  e = hipEventCreate(&b);
  if (e != hipSuccess) return e;
  (void)hipEventRecord(a, st);
  e = launch();
  (void)hipEventRecord(b, st);
  d.pending[k].push_back({a, b});
  return e;
}

hipError_t collect_times(Device& d) {
  for (int k = 0; k < Device::kKernels; ++k) {
    for (auto& pr : d.pending[k]) {
      hipError_t e = hipEventSynchronize(pr.second);
      if (e != hipSuccess) return e;
      float ms = 0;
      e = hipEventElapsedTime(&ms, pr.first, pr.second);
      if (e != hipSuccess) return e;
      d.acc_ms[k] += ms;
      d.launches[k] += 1;
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
    d.pending[k].clear();
  }
  return hipSuccess;
}

// ---- the armed latency kernel (verify_kernels.h k_ecdsa_wave_armed) ----
using pbftv::ArmArgs;
using pbftv::QcMail;
constexpr uint32_t kQcCap = QcMail::kQcCap;  // signatures per call the mailbox holds at its usual layout (= wide waves)

bool qc_arm_enabled() {
  const char* e = getenv("PBFTV_QC_ARM");
  return e ? e[0] == '1' : true;
}

double env_ms(const char* name, double dflt) {
  const char* e = getenv(name);
  return e ? atof(e) : dflt;
}

// How long one armed kernel waits for its request (PBFTV_QC_ARM_MS, default
// 100 ms; read at every arming), in wall-clock ticks of device dev.  A context
// that keeps making latency-path calls never sees a kernel run out: its keeper
// thread replaces the armed kernel at half its budget (qc_keeper_loop) for as
// long as the last call is less than PBFTV_QC_KEEP_MS (default 10 s) ago, so
// the reference's 1-s alarm cadence (pbft/network/node.go:44) finds one waiting.
// The budget bounds how long a hipDeviceSynchronize / hipFree made OUTSIDE the
// library on that GPU can wait for an armed kernel (~1.5 budgets).
double qc_arm_ms() { return env_ms("PBFTV_QC_ARM_MS", 100.0); }
double qc_keep_ms() { return env_ms("PBFTV_QC_KEEP_MS", 10000.0); }

uint64_t qc_arm_budget(int dev) {
  int khz = 100000;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  return (uint64_t)(qc_arm_ms() * khz);
}

// Whether the comb waves on a CU park while an armed workgroup there serves a
// certificate (PBFTV_QC_CU_YIELD: 1 the default, 0 never, 2 also on the CU
// that shares its instruction cache; verify_kernels.h comb_park)
uint32_t qc_cu_yield() {
  const char* e = getenv("PBFTV_QC_CU_YIELD");
  return e ? (uint32_t)atoi(e) : 1u;
}

// what the armed kernel does between polls (ArmArgs::spin; PBFTV_QC_SPIN)
uint32_t qc_spin() {
  const char* e = getenv("PBFTV_QC_SPIN");
  return e ? (uint32_t)atoi(e) : 0u;
}

// Whether an armed kernel yields to lane-path batches (PBFTV_QC_YIELD).  A
// kernel resident beside a busy stream costs it its wave slots: the narrow
// row server (4 workgroups) ~3 %, the wide one (a workgroup per signature of
// the largest recent wide certificate, 72 for 67 votes) 6-9 %
// (tools/armed_tax.py, profiles/r06_armed_tax_*.json).  A yielding server is
// halted by the batch enqueue (note_busy); a certificate in the meantime is
// launched on the free armed stream (one 128-VGPR wave per signature at
// raised priority, k_ecdsa_wave_lean: ~0.1 ms beside the batch instead of
// ~0.04 ms), and the keeper arms again once the queued batches are expected
// to be done.
//   "1": always yield;  "0": never (a server stays resident beside batches);
//   unset (the default): yield while certificates are sparse -- when none has
//   come for PBFTV_QC_YIELD_IDLE_MS (default 50 ms).  A node whose
//   certificates keep coming (every few ms) keeps its server resident beside
//   its flushes; one that checks a certificate now and then does not pay for
//   a resident server during every flush in between.
int qc_yield_mode() {
  const char* e = getenv("PBFTV_QC_YIELD");
  return e ? (e[0] == '1' ? 1 : 0) : 2;
}

bool qc_yield_now(const Device& d) {
  const int m = qc_yield_mode();
  if (m != 2) return m == 1;
  const auto idle = std::chrono::microseconds((int64_t)(env_ms("PBFTV_QC_YIELD_IDLE_MS", 50.0) * 1000.0));
  return std::chrono::steady_clock::now() - d.last_qc > idle;
}

// PBFTV_QC_SLOTS=k (1..kQcSlots): every narrow arming takes k slots; 0: unset
uint32_t qc_slots_fixed() {
  const char* e = getenv("PBFTV_QC_SLOTS");
  const int k = e ? atoi(e) : 0;
  return k >= 1 && k <= (int)QcMail::kQcSlots ? (uint32_t)k : 0u;
}

// per-certificate diagnostics on stderr (why a call was launched, a server
// that left unserved, the 2-s timeout): PBFTV_TRACE_QC=1, a switch of its own
// (PBFTV_TRACE, which bench.py sets for the registration phases, must not put
// stderr writes on the latency path)
bool trace_qc_enabled() {
  static const bool on = [] {
    const char* e = getenv("PBFTV_TRACE_QC");
    return e && e[0] == '1';
  }();
  return on;
}

int64_t steady_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

bool lane_busy(const Device& d) { return d.busy_until_ns.load(std::memory_order_relaxed) > steady_ns(); }

QcMail* qc_mail(Device& d) { return d.stage.as<QcMail>(); }

// the mailbox enters the process-wide registry (so a quiesce of its GPU halts
// its kernels) and leaves it before its memory is released
void qc_register(Device& d) {
  if (d.mail_registered || !d.stage.p) return;
  ArmRegistry& r = arm_registry();
  std::lock_guard<std::mutex> lk(r.mu);
  r.mail[d.id].push_back(qc_mail(d));
  r.keepers[d.id].push_back(&d.keeper_cv);
  d.mail_registered = true;
}

void qc_unregister(Device& d) {
  if (!d.mail_registered) return;
  ArmRegistry& r = arm_registry();
  std::lock_guard<std::mutex> lk(r.mu);
  auto& v = r.mail[d.id];
  v.erase(std::remove(v.begin(), v.end(), qc_mail(d)), v.end());
  auto& k = r.keepers[d.id];
  k.erase(std::remove(k.begin(), k.end(), &d.keeper_cv), k.end());
  d.mail_registered = false;
}

// (re)lay out the mailbox for up to cap signatures
hipError_t qc_mail_layout(Device& d, uint32_t cap) {
  if (d.stage.cap < QcMail::bytes(cap)) {
    qc_unregister(d);
    HIP_TRY_E(d.stage.ensure(QcMail::bytes(cap)));
  }
  std::memset(d.stage.p, 0, QcMail::bytes(cap));
  qc_mail(d)->cap = cap;
  qc_register(d);
  return hipSuccess;
}

hipError_t qc_mail_ready(Device& d) {
  if (d.stage.p && d.mail_registered) return hipSuccess;
  return qc_mail_layout(d, kQcCap);
}

// Cancel the armed kernels of this device (halt bump) and wait until they have exited.
hipError_t qc_disarm(Device& d) {
  if (d.stage.p && d.mail_registered) __atomic_add_fetch(&qc_mail(d)->halt, 1u, __ATOMIC_RELEASE);
  d.arm_seq = 0;
  d.retiring = 0;
  for (hipStream_t q : d.qstream)
    if (q) HIP_TRY_E(hipStreamSynchronize(q));
  return hipSuccess;
}

// Before a key change rewrites this context's key tables, key_valid or qptrs
// in place: nothing of THIS context may still read them.  Its armed kernels
// leave (qc_disarm), then its own streams drain, and every caller stream it
// was given: streams from pbftv_stream_create are known (stream_scratch); any
// other caller stream shares the device scratch, whose last use is fenced by
// scratch_ev, and every use waited for the one before it (scratch_acquire).
// Other contexts on the GPU are not waited for: their kernels read their own
// key tables, and a G table is never rewritten in place (a new width is a new
// table).  Frees inside the key change still quiesce the GPU (DevBuf).
hipError_t ctx_quiesce(Device& d) {
  HIP_TRY_E(qc_disarm(d));
  for (hipStream_t s : {d.stream, d.stream2, d.cstream, d.lstream})
    if (s) HIP_TRY_E(hipStreamSynchronize(s));
  for (auto& kv : d.stream_scratch) HIP_TRY_E(hipStreamSynchronize(kv.first));
  if (d.scratch_st && d.scratch_st != d.stream && d.scratch_ev) HIP_TRY_E(hipEventSynchronize(d.scratch_ev));
  for (auto& kv : d.reader_ev) HIP_TRY_E(hipEventSynchronize(kv.second));
  for (auto& kv : d.reader_ev) (void)hipEventDestroy(kv.second);
  d.reader_ev.clear();
  return hipSuccess;
}

// a verify that reads the key tables was just enqueued on st without the
// device scratch: fence it for the next key change if st is a caller stream
// the context does not know
hipError_t fence_reader(Device& d, hipStream_t st) {
#ifdef PBFTV_NO_READER_FENCE  // negative control for tests/test_gpu_keys_devices.py only
  return hipSuccess;
#endif
  if (st == d.stream || st == d.stream2 || d.stream_scratch.count(st)) return hipSuccess;
  if (d.reader_ev.size() >= 64 && !d.reader_ev.count(st)) {
    // a caller cycling through many streams: settle the fenced ones instead of
    // keeping an event per stream handle forever
    for (auto& kv : d.reader_ev) HIP_TRY_E(hipEventSynchronize(kv.second));
    for (auto& kv : d.reader_ev) (void)hipEventDestroy(kv.second);
    d.reader_ev.clear();
  }
  hipEvent_t& ev = d.reader_ev[st];
  if (!ev) HIP_TRY_E(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  return hipEventRecord(ev, st);
}

void qc_keeper_loop(Device* d);

// The armed kernels' two streams, at the HIGHEST priority: HIP keeps
// high-priority streams on hardware queues of their own (the normal ones are
// shared once a process has more streams than GPU_MAX_HW_QUEUES), and a
// kernel that stays resident on a normal-priority queue makes every
// synchronous null-stream operation on the GPU (hipMemcpy, a caller's or this
// library's) wait until it ends -- a full budget (tools/queue_share.hip,
// profiles/r05_queue_share.txt).  The CP also dispatches them first.
// Those queues are few (ArmRegistry::hiq_pairs): a context takes a pair only
// while the process holds fewer than GPU_MAX_HW_QUEUES / 2 on the GPU;
// otherwise it leaves qstream null (no armed server; latency_stream launches on
// lstream) and asks the holders' keepers to give one up.
int hiq_pair_cap() {
  static const int cap = [] {
    const char* e = getenv("GPU_MAX_HW_QUEUES");
    const int q = e && atoi(e) > 0 ? atoi(e) : 4;
    return q / 2;  // (one queue: no pair -- a successor would wait behind its predecessor)
  }();
  return cap;
}

// a context that found no pair free in the last second is waiting for one
constexpr auto kHiqWantedFor = std::chrono::seconds(1);
// a holder with no certificate for this long gives its pair to a waiting context
constexpr auto kHiqIdleGiveUp = std::chrono::milliseconds(200);

hipError_t qc_streams_ready(Device& d) {
  if (d.qstream[0] && d.qstream[1]) return hipSuccess;
  {
    ArmRegistry& r = arm_registry();
    std::lock_guard<std::mutex> lk(r.mu);
    if (r.hiq_pairs[d.id] >= hiq_pair_cap()) {
      r.hiq_wanted[d.id] = std::chrono::steady_clock::now();
      for (std::condition_variable* cv : r.keepers[d.id]) cv->notify_one();  // (qc_keeper_loop)
      return hipSuccess;
    }
    ++r.hiq_pairs[d.id];
    r.hiq_wanted.erase(d.id);  // (served; another waiter asks again at its next call)
  }
  for (hipStream_t& q : d.qstream) {
    int lo = 0, hi = 0;
    const char* pe = getenv("PBFTV_QC_PRIO");  // (experiments) "0": normal-priority armed streams
    hipError_t e = hipSuccess;
    if ((pe && pe[0] == '0') || hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
        hipStreamCreateWithPriority(&q, hipStreamNonBlocking, hi) != hipSuccess)
      e = hipStreamCreateWithFlags(&q, hipStreamNonBlocking);
    if (e != hipSuccess) {
      for (hipStream_t& p : d.qstream)
        if (p) {
          (void)hipStreamDestroy(p);
          p = nullptr;
        }
      ArmRegistry& r = arm_registry();
      std::lock_guard<std::mutex> lk(r.mu);
      --r.hiq_pairs[d.id];
      return e;
    }
  }
  d.arm_stream = 1;  // (the first arming takes qstream[0])
  return hipSuccess;
}

// Give the pair back: the armed kernels leave first (qc_disarm), then the
// streams go; the next call that arms claims a pair again.
hipError_t qc_streams_release(Device& d) {
  if (!d.qstream[0]) return hipSuccess;
  HIP_TRY_E(qc_disarm(d));
  for (hipStream_t& q : d.qstream) {
    (void)hipStreamDestroy(q);
    q = nullptr;
  }
  ArmRegistry& r = arm_registry();
  std::lock_guard<std::mutex> lk(r.mu);
  --r.hiq_pairs[d.id];
  return hipSuccess;
}

// whether another context on this GPU asked for a pair lately
bool hiq_wanted(const Device& d, std::chrono::steady_clock::time_point now) {
  ArmRegistry& r = arm_registry();
  std::lock_guard<std::mutex> lk(r.mu);
  auto it = r.hiq_wanted.find(d.id);
  return it != r.hiq_wanted.end() && now - it->second < kHiqWantedFor;
}

// Where a latency-path kernel is LAUNCHED (a certificate the armed server
// cannot take, its exact rerun, a small digest call): the armed stream that
// holds no resident kernel -- a hardware queue of its own, never behind a
// batch (a normal stream may share its hardware queue with the stream the
// batches are queued on), dispatched first; the next arming queues behind the
// short launched kernel.  While a rotation keeps both armed streams resident,
// or while the context holds no pair (hiq_pair_cap), the normal-priority
// latency stream (lstream).  No extra high-priority
// stream: their hardware queues are few too, and a stream sharing one with a
// resident armed kernel would wait for that kernel's budget.
hipError_t latency_stream(Device& d, hipStream_t* out) {
  HIP_TRY_E(qc_streams_ready(d));
  if (d.qstream[0] && !d.arm_seq) {
    *out = d.qstream[0];
  } else if (d.qstream[0] && !d.retiring) {
    *out = d.qstream[d.arm_stream ^ 1];
  } else {
    if (!d.lstream) HIP_TRY_E(hipStreamCreateWithFlags(&d.lstream, hipStreamNonBlocking));
    *out = d.lstream;
  }
  return hipSuccess;
}

// arm the wide kernel (kQcCap waves) while calls of 9..kQcCap signatures keep
// coming (PBFTV_QC_KEEP_MS since the last one; PBFTV_QC_WIDE=0: never).  Its
// 120 helper waves hold ~half a SIMD of registers each while armed, so a
// context that only sees small certificates keeps the narrow kernel.
// PBFTV_QC_WIDE: "0" never arm the wide kernel (wide certificates are
// launched), "split" never either, but split a wide certificate between the
// armed narrow slots and one launch; unset or "1": arm the wide kernel
int qc_wide_mode() {
  const char* e = getenv("PBFTV_QC_WIDE");
  if (!e) return 1;
  return e[0] == '0' ? 0 : e[0] == 's' ? 2 : 1;
}

bool qc_wide_wanted(const Device& d) {
  if (qc_wide_mode() != 1) return false;
  if (d.last_wide.time_since_epoch().count() == 0) return false;
  return std::chrono::steady_clock::now() - d.last_wide < std::chrono::microseconds((int64_t)(qc_keep_ms() * 1000.0));
}

// Launch the kernel that will serve the next latency-path request (none while
// a quiesce of this GPU is in progress: the request then takes a launch).
hipError_t qc_arm(Device& d) {
  if (d.arm_seq || !qc_arm_enabled() || !d.have_keys) return hipSuccess;
  if (qc_yield_now(d) && lane_busy(d)) return hipSuccess;  // the keeper arms once the batches are done
  HIP_TRY_E(qc_mail_ready(d));
  HIP_TRY_E(qc_streams_ready(d));
  if (!d.qstream[0]) return hipSuccess;  // no high-priority pair free: certificates are launched
  uint32_t halt;
  {
    // the check and the halt snapshot in one critical section: a quiesce that
    // starts after it bumps halt, and the new kernel leaves at its first poll
    ArmRegistry& r = arm_registry();
    std::lock_guard<std::mutex> lk(r.mu);
    if (!arming_allowed_locked(r, d.id)) return hipSuccess;
    halt = __atomic_load_n(&qc_mail(d)->halt, __ATOMIC_ACQUIRE);
  }
  if (++d.seq_counter == 0) d.seq_counter = 1;  // 0 means "none armed"
  const uint32_t want = d.seq_counter;
  const int slot = d.arm_stream ^ 1;  // not behind the previous armed kernel (a rotation overlaps the two)
  uint64_t* relay = nullptr;
  if (qc_wide_wanted(d)) {  // certificates of 9..kQcCap signatures were seen lately: helpers for them
    d.qrelay.flags = hipDeviceMallocUncached;
    HIP_TRY_E(d.qrelay.ensure(128));
    relay = reinterpret_cast<uint64_t*>(d.qrelay.as<uint8_t>() + 64 * slot);
    HIP_TRY_E(hipMemsetAsync(relay, 0, 8, d.qstream[slot]));  // after that stream's previous kernel left
  }
  // Narrow slots: the row schedule's armed kernel holds one CU per slot, so it
  // arms as many as the largest certificate of the last period (kept while no
  // call came), at least 4 (a 3-vote certificate of a 4-replica committee, the
  // reference's default, and its 4-vote form); a larger one is served by a
  // launch and re-arms wider at once.  PBFTV_QC_SLOTS=k fixes k (1..8).
  // (the largest of the last two periods with calls: mixed sizes, say 7- and
  // 3-vote certificates, keep the wider arming instead of falling back to a
  // launch after every half-budget rotation)
  if (d.qc_nmax) {
    d.qc_slots = std::max({4u, d.qc_nmax, d.qc_nmax_prev});
    d.qc_nmax_prev = d.qc_nmax;
  }
  d.qc_nmax = 0;
  const char* re = getenv("PBFTV_QC_ROWS");
  uint32_t slots = (re && re[0] == '0') ? QcMail::kQcSlots : d.qc_slots;
  if (const uint32_t k = qc_slots_fixed()) slots = k;
  // wide: one workgroup per signature of the largest certificate seen while
  // wide ones keep coming, rounded up to 8 (a 67-vote certificate arms 72, not
  // 128 -- the resident footprint is ~6 waves per workgroup); a larger one is
  // launched once and the next arming is wider; it never shrinks until wide
  // certificates stop (qc_wide_wanted)
  if (relay) {
    if (d.qc_wmax) d.qc_wslots = std::max(d.qc_wslots, std::min<uint32_t>(kQcCap, (d.qc_wmax + 7) / 8 * 8));
    if (!d.qc_wslots) d.qc_wslots = kQcCap;
  } else {
    d.qc_wslots = 0;
  }
  d.qc_wmax = 0;
  const uint32_t wslots = (re && re[0] == '0') ? kQcCap : d.qc_wslots;
  const char* se = getenv("PBFTV_QC_STAMPS");
  const uint32_t cuyield = qc_cu_yield();
  if (cuyield && !d.cuflag.p) {  // zeroed before any kernel reads or writes it
    HIP_TRY_E(d.cuflag.ensure(4 * pbftv::kCuFlagWords));
    HIP_TRY_E(hipMemsetAsync(d.cuflag.p, 0, 4 * pbftv::kCuFlagWords, d.qstream[slot]));
    HIP_TRY_E(hipStreamSynchronize(d.qstream[slot]));
    d.cuflag_ready.store(d.cuflag.as<uint32_t>(), std::memory_order_release);
  }
  const ArmArgs a{qc_mail(d),
                  want,
                  qc_arm_budget(d.id),
                  d.key_valid.as<uint32_t>(),
                  d.nkeys,
                  d.gtab->as<uint32_t>(),
                  d.qptrs.as<const uint32_t* const>(),
                  qc_spin(),
                  halt,
                  relay,
                  se && se[0] == '1' ? 1u : 0u,
                  slot,
                  relay ? wslots : slots,
                  cuyield ? d.cuflag.as<uint32_t>() : nullptr,
                  cuyield};
  HIP_TRY_E(pbftv::launch_ecdsa_wave_armed(d.gbits, d.qbits, a, d.qstream[slot]));
  d.arm_seq = d.armed_first = want;
  d.arm_waves = relay ? wslots : slots;
  d.arm_wide = relay != nullptr;
  d.arm_live = false;
  ++d.qc_armings;
  d.arm_stream = slot;
  d.armed_at = std::chrono::steady_clock::now();
  if (!d.keeper.joinable() && qc_keep_ms() > 0) d.keeper = std::thread(qc_keeper_loop, &d);
  d.keeper_cv.notify_one();
  return hipSuccess;
}

// Replace the armed kernel before it runs out: the successor is launched on
// the other stream; the old one keeps serving nothing but stays resident until
// the successor reports itself live (its waves may wait for free slots behind
// a large batch), then the keeper retires it (stop = its number).  No request
// is in flight meanwhile: both run under d.mu.
hipError_t qc_rotate(Device& d) {
  const uint32_t old = d.arm_seq;
  d.arm_seq = 0;
  hipError_t e = qc_arm(d);
  if (e != hipSuccess || d.arm_seq == 0) {  // not now (quiesce): the old one runs out
    d.arm_seq = old;
    return e;
  }
  if (old) {
    if (d.retiring) __atomic_store_n(&qc_mail(d)->stop, d.retiring, __ATOMIC_RELEASE);  // (not live yet: rare)
    d.retiring = old;
    if (d.arm_wide) {
      // a wide successor (up to 128 workgroups of ~6 waves) may not find room
      // beside its predecessor -- and beside other contexts' servers -- so
      // the predecessor leaves at once instead of overlapping (a wide
      // certificate in the gap is launched: qc_all_live)
      __atomic_store_n(&qc_mail(d)->stop, old, __ATOMIC_RELEASE);
      d.retiring = 0;
    }
  }
  return hipSuccess;
}

// every workgroup of the armed kernel resident (checked once per arming)
bool qc_all_live(Device& d) {
  if (d.arm_live) return true;
  if (!d.arm_seq) return false;
  const uint32_t* live = reinterpret_cast<const uint32_t*>(d.stage.as<uint8_t>() + QcMail::live_off(d.arm_stream));
  for (uint32_t w = 0; w < d.arm_waves; ++w)
    if (__atomic_load_n(live + w, __ATOMIC_ACQUIRE) != d.armed_first) return false;
  d.arm_live = true;
  return true;
}

// retire the rotated-out kernel once its successor is resident
// (its slot workgroups, <= kQcSlots: a wide successor's helpers may find room
// only once the predecessor has left -- two wide row kernels need up to 256
// workgroups of ~6 waves -- and until they are all resident a wide
// certificate is launched, qc_all_live)
void qc_retire(Device& d) {
  if (!d.retiring || !d.arm_seq) return;
  const uint32_t* live = reinterpret_cast<const uint32_t*>(d.stage.as<uint8_t>() + QcMail::live_off(d.arm_stream));
  for (uint32_t w = 0; w < std::min<uint32_t>(d.arm_waves, QcMail::kQcSlots); ++w)
    if (__atomic_load_n(live + w, __ATOMIC_ACQUIRE) != d.armed_first) return;  // not every slot resident yet
  __atomic_store_n(&qc_mail(d)->stop, d.retiring, __ATOMIC_RELEASE);
  d.retiring = 0;
}

// One per device with a latency path in use: keeps an armed kernel waiting
// while calls keep coming (PBFTV_QC_KEEP_MS after the last one), so a call
// after an idle gap longer than the budget still finds one.
void qc_keeper_loop(Device* d) {
  std::unique_lock<std::mutex> lk(d->mu);
  (void)hipSetDevice(d->id);
  const auto far = std::chrono::hours(1);
  while (!d->keeper_stop) {
    const auto now = std::chrono::steady_clock::now();
    const auto half = std::chrono::microseconds((int64_t)(qc_arm_ms() * 500.0));
    const auto keep = std::chrono::microseconds((int64_t)(qc_keep_ms() * 1000.0));
    auto wake = now + far;
    qc_retire(*d);
    // another context on this GPU is waiting for a high-priority pair
    // (qc_streams_ready): ours goes to it once no certificate came here for
    // kHiqIdleGiveUp; our next call claims one again
    if (d->qstream[0] && hiq_wanted(*d, now)) {
      if (now - d->last_qc >= kHiqIdleGiveUp) {
        if (qc_streams_release(*d) != hipSuccess) (void)hipGetLastError();
        d->qstream_given_up = now;
      } else {
        wake = d->last_qc + kHiqIdleGiveUp;
      }
    }
    const bool given_up = !d->qstream[0] && d->last_qc <= d->qstream_given_up;  // (no call since: nothing to arm)
    const bool wanted = !given_up && qc_arm_enabled() && d->have_keys && now - d->last_qc < keep;
    const int64_t busy_ns = d->busy_until_ns.load(std::memory_order_relaxed) - steady_ns();
    if (wanted && qc_yield_now(*d) && busy_ns > 0) {
      // lane-path batches are queued: nothing armed until they are expected done
      wake = std::min(wake, now + std::chrono::nanoseconds(busy_ns + 50000));
    } else if (wanted) {
      // also re-arms after a disarm (key change) or a halt (quiesce)
      // (the kernel's SHAPE, narrow or wide, not its size: a wide arming takes
      // as many workgroups as the largest recent wide certificate)
      const bool reshape = d->arm_seq && d->arm_wide != qc_wide_wanted(*d);
      const bool left = d->arm_seq && __atomic_load_n(qc_mail(*d)->expired(d->arm_stream), __ATOMIC_ACQUIRE) == d->arm_seq;
      if (d->arm_seq == 0 || now >= d->armed_at + half || reshape || left) {  // (left: halted by a quiesce)
        if (qc_rotate(*d) != hipSuccess) (void)hipGetLastError();  // a call will launch instead
        ++d->rotations;
      }
      wake = std::min(wake, d->arm_seq            ? std::min(d->armed_at + half, d->last_qc + keep)
                            : d->qstream[0] ? now + std::chrono::milliseconds(1)
                                            : now + std::chrono::milliseconds(50));  // (no pair free: retry)
    }
    if (d->retiring) wake = std::min(wake, now + std::chrono::microseconds(100));  // (a wide successor waits for its room)
    if (wake <= now) wake = now + std::chrono::milliseconds(1);
    d->keeper_idle = wake - now > std::chrono::minutes(1);  // a call wakes it (d.last_qc moved)
    d->keeper_cv.wait_until(lk, wake);
  }
}

// stop the keeper (not under d.mu)
void qc_keeper_stop(Device& d) {
  {
    std::lock_guard<std::mutex> lk(d.mu);
    d.keeper_stop = true;
  }
  d.keeper_cv.notify_one();
  if (d.keeper.joinable()) d.keeper.join();
}

}  // namespace

// G comb tables by (HIP device, width): built once and shared by every
// context (and aliased logical device) on that GPU while one holds it.
// g_tables_mu guards the map only; a table is built under its own slot's
// build mutex, so GPUs build their G tables in parallel and lookups of other
// widths or devices never wait for a build.
struct GSlot {
  std::weak_ptr<DevBuf> tab;
  std::shared_ptr<std::mutex> build = std::make_shared<std::mutex>();
};
std::mutex g_tables_mu;
std::map<std::pair<int, int>, GSlot> g_tables;

struct pbftv_ctx {
  std::vector<std::unique_ptr<Device>> devs;
  bool timing = false;
  // batches up to this size take the latency path (PBFTV_WAVE_MAX at open,
  // pbftv_set_latency_path_max): read once, not per call (a cold getenv cost
  // a certificate ~3 us after an idle second)
  std::atomic<uint64_t> wave_max{2048};
  Device* dev0 = nullptr;  // devs[0], one hop less for the latency path's first (cold) loads
  // pbftv_host_alloc / pbftv_host_free: freed pinned blocks are kept for
  // reuse (hipHostFree waits for every kernel on every GPU, so a free would
  // halt the armed servers); released at close, or when the cache passes
  // kHostCacheBytes (then under a quiesce)
  std::mutex host_mu;
  std::map<void*, size_t> host_live;          // block -> its size
  std::multimap<size_t, void*> host_cache;    // size -> free block
  size_t host_cache_bytes = 0;
  static constexpr size_t kHostCacheBytes = size_t(1) << 30;
};

namespace {

constexpr uint64_t kShardAlign = 512;


struct Shard {
  uint64_t lo, hi;
};

std::vector<Shard> plan_shards(uint64_t n, size_t ndev) {
  std::vector<Shard> out;
  if (n == 0) return out;
  uint64_t per = (n + ndev - 1) / ndev;
  per = (per + kShardAlign - 1) / kShardAlign * kShardAlign;
  for (uint64_t lo = 0; lo < n; lo += per) out.push_back({lo, std::min(n, lo + per)});
  return out;
}

// run fn(dev, shard) on every shard; one host thread per device when > 1 shard
template <class Fn>
int run_sharded(pbftv_ctx* ctx, uint64_t n, Fn fn) {
  auto shards = plan_shards(n, ctx->devs.size());
  if (shards.size() <= 1) {
    return shards.empty() ? PBFTV_OK : fn(*ctx->devs[0], shards[0]);
  }
  std::vector<int> rc(shards.size(), PBFTV_OK);
  std::vector<std::string> errs(shards.size());
  std::vector<std::thread> th;
  for (size_t s = 0; s < shards.size(); ++s) {
    th.emplace_back([&, s] {
      rc[s] = fn(*ctx->devs[s], shards[s]);
      if (rc[s] != PBFTV_OK) errs[s] = g_last_error;
    });
  }
  for (auto& t : th) t.join();
  for (size_t s = 0; s < shards.size(); ++s)
    if (rc[s] != PBFTV_OK) return fail(rc[s], errs[s]);
  return PBFTV_OK;
}

hipStream_t pick_stream(Device& d, void* stream) { return stream ? reinterpret_cast<hipStream_t>(stream) : d.stream; }

// ---- message batches: column inputs packed for ONE host->device copy ----
// Host segments are copied (16-B aligned) into the device's pinned staging
// buffer, then to its device arena with a single hipMemcpyAsync.
struct Packer {
  struct Seg {
    const void* src;
    size_t bytes, off;
  };
  std::vector<Seg> segs;
  std::vector<std::vector<uint64_t>> owned;  // rebased offsets, slots (inner buffers stay put when moved)
  size_t total = 0;
  bool null_blob = false;  // a string column with nonzero lengths but no data pointer
  size_t add(const void* src, size_t bytes) {
    const size_t o = total;
    segs.push_back({src, bytes, o});
    total = (o + bytes + 15) & ~(size_t)15;
    return o;
  }
  size_t add_owned(std::vector<uint64_t>&& v) {
    owned.push_back(std::move(v));
    return add(owned.back().data(), owned.back().size() * 8);
  }
  // string column restricted to items [lo, hi): the blob span they use, offsets rebased onto it
  struct Str {
    size_t data, off, len;
  };
  Str add_str(const uint8_t* data, const uint64_t* off, const uint32_t* len, uint64_t lo, uint64_t hi) {
    uint64_t a = UINT64_MAX, b = 0;
    for (uint64_t i = lo; i < hi; ++i)
      if (len[i]) {
        a = std::min(a, off[i]);
        b = std::max(b, off[i] + len[i]);
      }
    if (a > b) a = b = 0;
    if (b > a && data == nullptr) {
      null_blob = true;
      a = b = 0;
    }
    std::vector<uint64_t> r(hi - lo);
    for (uint64_t i = lo; i < hi; ++i) r[i - lo] = len[i] ? off[i] - a : 0;
    Str s;
    s.data = add(b > a ? data + a : nullptr, b - a);
    s.off = add_owned(std::move(r));
    s.len = add(len + lo, 4 * (hi - lo));
    return s;
  }
};

// pinned copy + one H2D into d.arena (stream-ordered before the kernels that read it)
int upload(Device& d, const Packer& p) {
  if (p.null_blob) return fail(PBFTV_EINVAL, "string column: nonzero lengths with a null data pointer");
  HIP_TRY(d.mstage.ensure(p.total + 16));
  HIP_TRY(d.arena.ensure(p.total + 16));
  uint8_t* h = d.mstage.as<uint8_t>();
  for (const auto& s : p.segs)
    if (s.bytes) std::memcpy(h + s.off, s.src, s.bytes);
  if (p.total) HIP_TRY(hipMemcpyAsync(d.arena.p, h, p.total, hipMemcpyHostToDevice, d.stream));
  return PBFTV_OK;
}

template <class T>
const T* at(const Device& d, size_t off) {
  return reinterpret_cast<const T*>(d.arena.as<uint8_t>() + off);
}

pbftv::StrCol str_col(const Device& d, const Packer::Str& s) {
  return {at<uint8_t>(d, s.data), at<uint64_t>(d, s.off), at<uint32_t>(d, s.len)};
}

// slot offsets of the preimage buffer from per-item encoder bounds (4-B aligned)
template <class Bound>
std::vector<uint64_t> slots(uint64_t lo, uint64_t hi, Bound bound, uint64_t* total) {
  std::vector<uint64_t> s(hi - lo);
  uint64_t t = 0;
  for (uint64_t i = lo; i < hi; ++i) {
    s[i - lo] = t;
    t += (bound(i) + 3) & ~3ull;
  }
  *total = t;
  return s;
}

// encode (launch(slot_dev) writes preimages into d.data, lengths into
// d.lengths), then SHA-256 of every slot into d.digests
template <class Launch>
int encode_and_hash(Device& d, uint64_t m, const uint64_t* slot_dev, uint64_t pre_bytes, Launch launch) {
  HIP_TRY(d.data.ensure(pre_bytes + 64));
  HIP_TRY(d.lengths.ensure(m * 4 + 4));
  HIP_TRY(d.digests.ensure(m * 32 + 32));
  HIP_TRY(timed(d, PBFTV_K_GOJSON, d.stream, launch));
  HIP_TRY(timed(d, PBFTV_K_SHA256, d.stream, [&] {
    return pbftv::launch_sha256(d.data.as<uint8_t>(), slot_dev, d.lengths.as<uint32_t>(), nullptr, m,
                                d.digests.as<uint8_t>(), nullptr, nullptr, d.stream);
  }));
  return PBFTV_OK;
}

// Results of one flush shard [lo, lo + m), copied back in ONE device -> host
// round trip through pinned staging: 32-B digests, a device bitmap (tail bits
// past the shard masked), or one flag byte per item packed into bits.
enum OutKind { kDigests, kBitmap, kByteFlags };
struct OutSeg {
  OutKind kind;
  const void* dev;
  uint8_t* host;  // the caller's whole-batch buffer (null: not requested)
};

int results_out(Device& d, uint64_t lo, uint64_t m, std::initializer_list<OutSeg> segs) {
  const uint64_t nb = (m + 7) / 8;
  auto bytes = [&](OutKind k) -> uint64_t { return k == kDigests ? 32 * m : (k == kBitmap ? nb : m); };
  size_t total = 0;
  for (const auto& g : segs)
    if (g.host) total += (bytes(g.kind) + 15) & ~(uint64_t)15;
  if (total == 0) return PBFTV_OK;
  HIP_TRY(d.mout.ensure(total + 16));
  uint8_t* h = d.mout.as<uint8_t>();
  size_t off = 0;
  for (const auto& g : segs) {
    if (!g.host) continue;
    HIP_TRY(hipMemcpyAsync(h + off, g.dev, bytes(g.kind), hipMemcpyDeviceToHost, d.stream));
    off += (bytes(g.kind) + 15) & ~(uint64_t)15;
  }
  HIP_TRY(hipStreamSynchronize(d.stream));
  off = 0;
  for (const auto& g : segs) {
    if (!g.host) continue;
    const uint8_t* src = h + off;
    if (g.kind == kDigests) {
      std::memcpy(g.host + 32 * lo, src, 32 * m);
    } else if (g.kind == kBitmap) {
      std::memcpy(g.host + lo / 8, src, nb);
      if (m % 8) g.host[lo / 8 + nb - 1] &= (uint8_t)((1u << (m % 8)) - 1u);
    } else {
      uint8_t* bm = g.host + lo / 8;
      std::memset(bm, 0, nb);
      for (uint64_t i = 0; i < m; ++i) bm[i >> 3] |= (uint8_t)((src[i] & 1u) << (i & 7));
    }
    off += (bytes(g.kind) + 15) & ~(uint64_t)15;
  }
  return PBFTV_OK;
}

// the same slot layout twice: a second preimage set right after the first
std::vector<uint64_t> twice(std::vector<uint64_t> s, uint64_t* total) {
  const size_t m = s.size();
  s.resize(2 * m);
  for (size_t i = 0; i < m; ++i) s[m + i] = s[i] + *total;
  *total *= 2;
  return s;
}

bool keys_ready(pbftv_ctx* ctx) {
  for (auto& dp : ctx->devs)
    if (!dp->have_keys) return false;
  return true;
}

}  // namespace

extern "C" {

const char* pbftv_strerror(int code) {
  switch (code) {
    case PBFTV_OK: return "ok";
    case PBFTV_EINVAL: return "invalid argument";
    case PBFTV_ENODEV: return "no usable gfx950 device";
    case PBFTV_EDEVICE: return "HIP device error";
    case PBFTV_ENOMEM: return "out of memory";
    case PBFTV_ENOKEYS: return "no keys registered";
    default: return "unknown error";
  }
}

const char* pbftv_last_error(void) { return g_last_error.c_str(); }

int pbftv_open(pbftv_ctx** out, uint32_t device_mask) {
  if (!out) return fail(PBFTV_EINVAL, "out is null");
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return fail(PBFTV_ENODEV, "no HIP devices visible");
  auto ctx = std::make_unique<pbftv_ctx>();
  // PBFTV_ALIAS_DEVICES=k (tests only): k logical devices per GPU, each with its
  // own stream, tables and scratch -- the multi-device paths (shards, per-device
  // registration, bitmap concatenation) on a one-GPU machine.
  int alias = 1;
  if (const char* e = getenv("PBFTV_ALIAS_DEVICES")) alias = std::min(8, std::max(1, atoi(e)));
  for (int d = 0; d < count && d < 32; ++d) {
    if (device_mask && !((device_mask >> d) & 1u)) continue;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d) != hipSuccess) continue;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) continue;  // the kernels are gfx950 code objects
    for (int a = 0; a < alias; ++a) {
      auto dev = std::make_unique<Device>();
      dev->id = d;
      dev->timing = &ctx->timing;
      dev->wave_max = &ctx->wave_max;
      HIP_TRY(hipSetDevice(d));
      HIP_TRY(hipStreamCreateWithFlags(&dev->stream, hipStreamNonBlocking));
      ctx->devs.push_back(std::move(dev));
    }
  }
  if (ctx->devs.empty()) return fail(PBFTV_ENODEV, "no gfx950 device in device_mask");
  ctx->dev0 = ctx->devs[0].get();
  ctx->wave_max = pbftv::wave_path_max();
  *out = ctx.release();
  return PBFTV_OK;
}

void pbftv_close(pbftv_ctx* ctx) {
  if (!ctx) return;
  for (auto& d : ctx->devs) qc_keeper_stop(*d);
  for (auto& d : ctx->devs) {
    std::lock_guard<std::mutex> lk(d->mu);
    (void)hipSetDevice(d->id);
    (void)qc_disarm(*d);  // the armed latency kernels exit before anything is freed
    qc_unregister(*d);
    (void)qc_streams_release(*d);
    (void)hipStreamSynchronize(d->stream);
    (void)collect_times(*d);
    for (auto& b : d->qblocks) b->release();
    for (auto& b : d->tab_scratch) b.release();
    d->tab_keys.release();
    d->gtab.reset();
    d->vs.release();
    for (DevBuf* b : {&d->qptrs, &d->key_valid, &d->hashes, &d->sigs, &d->key_idx,
                      &d->bitmap, &d->data, &d->offsets, &d->lengths, &d->order,
                      &d->order_scratch, &d->digests, &d->expected, &d->shabits, &d->arena, &d->msgok, &d->cuflag})
      b->release();  // explicit, with this device current (the destructors are a backstop)
    d->cuflag_ready.store(nullptr);
    for (HostBuf* b : {&d->stage, &d->mstage, &d->mout, &d->sstage}) b->release();
    if (d->scratch_ev) (void)hipEventDestroy(d->scratch_ev);
    for (auto& kv : d->reader_ev) (void)hipEventDestroy(kv.second);
    d->reader_ev.clear();
    if (d->stream2) {
      (void)hipStreamSynchronize(d->stream2);
      (void)hipStreamDestroy(d->stream2);
    }
    if (d->lstream) {
      (void)hipStreamSynchronize(d->lstream);
      (void)hipStreamDestroy(d->lstream);
    }
    d->vs2.release();
    for (auto& kv : d->stream_scratch) {  // streams the caller did not destroy: their scratch
      (void)hipStreamSynchronize(kv.first);
      kv.second->release();
    }
    d->stream_scratch.clear();
    if (d->join_ev) (void)hipEventDestroy(d->join_ev);
    d->keys_all.release();
    if (d->cstream) {
      (void)hipStreamSynchronize(d->cstream);
      (void)hipStreamDestroy(d->cstream);
    }
    for (int k = 0; k < Device::kSlots; ++k) {
      d->din[k].release();
      if (d->h2d_ev[k]) (void)hipEventDestroy(d->h2d_ev[k]);
      if (d->comp_ev[k]) (void)hipEventDestroy(d->comp_ev[k]);
    }
    if (d->pool) {  // pending frees and blocks the caller did not free go with the context
      GpuQuiesce quiet(d->id);
      for (auto& pf : d->pending_frees) {
        for (hipEvent_t e : pf.ev) {
          (void)hipEventSynchronize(e);
          d->spare_ev.push_back(e);
        }
        (void)hipFreeAsync(pf.p, d->astream);
      }
      d->pending_frees.clear();
      for (void* p : d->pool_ptrs) (void)hipFreeAsync(p, d->astream);
      d->pool_ptrs.clear();
      (void)hipStreamSynchronize(d->astream);
      (void)hipMemPoolDestroy(d->pool);
      (void)hipStreamDestroy(d->astream);
    }
    for (hipEvent_t e : d->spare_ev) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(d->stream);
  }
  if (!ctx->host_cache.empty()) {
    GpuQuiesce quiet(-1);
    for (auto& kv : ctx->host_cache) (void)hipHostFree(kv.second);
  }
  delete ctx;
}

int pbftv_device_count(const pbftv_ctx* ctx) { return ctx ? (int)ctx->devs.size() : 0; }

int pbftv_device_id(const pbftv_ctx* ctx, int i) {
  if (!ctx || i < 0 || i >= (int)ctx->devs.size()) return -1;
  return ctx->devs[i]->id;
}

int pbftv_reserve(pbftv_ctx* ctx, uint64_t n) {
  if (!ctx) return fail(PBFTV_EINVAL, "ctx is null");
  for (auto& dp : ctx->devs) {
    Device& d = *dp;
    std::lock_guard<std::mutex> lk(d.mu);
    HIP_TRY(hipSetDevice(d.id));
    HIP_TRY(d.vs.rec.ensure(pbftv::ecdsa_record_bytes(n)));
    HIP_TRY(d.vs.prefix.ensure(pbftv::scalar_prefix_bytes(n)));
    if (pbftv::key_sort_wanted(n, d.nkeys)) {
      HIP_TRY(ensure_key_sort(d.vs, n, d.nkeys, nullptr));
      HIP_TRY(d.vs.okb.ensure(n));
    }
  }
  return PBFTV_OK;
}

// ---------------------------------------------------------------- plumbing
static Device* dev_of(pbftv_ctx* ctx, int dev) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return nullptr;
  return ctx->devs[dev].get();
}

// The device pool of pbftv_dev_alloc: memory is never returned to the
// driver while the context lives (release threshold: unlimited), so a free
// is bookkeeping, not hipFree (which waits for every kernel on the GPU, the
// armed servers included).  Allocations are made on astream and reuse only
// blocks whose free has completed (no reuse that would make an allocation
// wait for a pending free).
static hipError_t dev_pool_ready(Device& d) {
  if (d.pool) return hipSuccess;
  hipMemPoolProps props{};
  props.allocType = hipMemAllocationTypePinned;
  props.handleTypes = hipMemHandleTypeNone;
  props.location.type = hipMemLocationTypeDevice;
  props.location.id = d.id;
  HIP_TRY_E(hipMemPoolCreate(&d.pool, &props));
  uint64_t keep = UINT64_MAX;
  HIP_TRY_E(hipMemPoolSetAttribute(d.pool, hipMemPoolAttrReleaseThreshold, &keep));
  int no = 0;
  HIP_TRY_E(hipMemPoolSetAttribute(d.pool, hipMemPoolReuseAllowInternalDependencies, &no));
  HIP_TRY_E(hipMemPoolSetAttribute(d.pool, hipMemPoolReuseFollowEventDependencies, &no));
  HIP_TRY_E(hipStreamCreateWithFlags(&d.astream, hipStreamNonBlocking));
  return hipSuccess;
}

// A free: events on the context's own streams and its library streams
// (pbftv_stream_create) mark what may still use the block; no stream waits
// for them (a wait packet would stall every stream sharing that stream's
// hardware queue).  Work the context put on CALLER streams (the scratch fence
// and the reader fences of *_dev calls on streams it did not create) is waited
// for on the host here, as hipFree's implicit synchronisation would -- only
// that work, not the whole GPU.
static hipError_t defer_free(Device& d, void* p) {
  if (d.scratch_st && d.scratch_st != d.stream && !d.stream_scratch.count(d.scratch_st) && d.scratch_ev)
    HIP_TRY_E(hipEventSynchronize(d.scratch_ev));
  for (auto& kv : d.reader_ev) HIP_TRY_E(hipEventSynchronize(kv.second));
  Device::PendingFree pf{p, {}};
  auto mark = [&](hipStream_t st) -> hipError_t {
    hipEvent_t e;
    if (!d.spare_ev.empty()) {
      e = d.spare_ev.back();
      d.spare_ev.pop_back();
    } else {
      HIP_TRY_E(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    pf.ev.push_back(e);
    return hipEventRecord(e, st);
  };
  for (hipStream_t st : {d.stream, d.stream2, d.cstream, d.lstream})
    if (st) HIP_TRY_E(mark(st));
  for (auto& kv : d.stream_scratch) HIP_TRY_E(mark(kv.first));
  d.pending_frees.push_back(std::move(pf));
  return hipSuccess;
}

// return the blocks whose marks have all passed to the pool (host polls)
static hipError_t reap_frees(Device& d) {
  size_t k = 0;
  for (auto& pf : d.pending_frees) {
    bool done = true;
    for (hipEvent_t e : pf.ev) {
      const hipError_t q = hipEventQuery(e);
      if (q == hipErrorNotReady) {
        done = false;
        break;
      }
      if (q != hipSuccess) return q;
    }
    if (!done) {
      d.pending_frees[k++] = std::move(pf);
      continue;
    }
    for (hipEvent_t e : pf.ev) d.spare_ev.push_back(e);
    HIP_TRY_E(hipFreeAsync(pf.p, d.astream));
  }
  d.pending_frees.resize(k);
  return hipSuccess;
}

int pbftv_dev_alloc(pbftv_ctx* ctx, int dev, uint64_t bytes, void** out_ptr) {
  Device* d = dev_of(ctx, dev);
  if (!d || !out_ptr) return fail(PBFTV_EINVAL, "bad context, device index or out pointer");
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  HIP_TRY(dev_pool_ready(*d));
  HIP_TRY(reap_frees(*d));
  HIP_TRY(hipMallocFromPoolAsync(out_ptr, bytes ? bytes : 1, d->pool, d->astream));
  HIP_TRY(hipStreamSynchronize(d->astream));  // (usable on any stream once this returns)
  d->pool_ptrs.insert(*out_ptr);
  return PBFTV_OK;
}

int pbftv_host_alloc(pbftv_ctx* ctx, uint64_t bytes, void** out_ptr) {
  if (!ctx || !out_ptr || ctx->devs.empty()) return fail(PBFTV_EINVAL, "bad context or out pointer");
  const size_t want = bytes ? bytes : 1;
  {
    // a cached block of at least the size and at most twice it
    std::lock_guard<std::mutex> lk(ctx->host_mu);
    auto it = ctx->host_cache.lower_bound(want);
    if (it != ctx->host_cache.end() && it->first <= 2 * want) {
      *out_ptr = it->second;
      ctx->host_live[it->second] = it->first;
      ctx->host_cache_bytes -= it->first;
      ctx->host_cache.erase(it);
      return PBFTV_OK;
    }
  }
  HIP_TRY(hipSetDevice(ctx->devs[0]->id));
  HIP_TRY(hipHostMalloc(out_ptr, want, hipHostMallocPortable));
  std::lock_guard<std::mutex> lk(ctx->host_mu);
  ctx->host_live[*out_ptr] = want;
  return PBFTV_OK;
}

int pbftv_host_free(pbftv_ctx* ctx, void* ptr) {
  if (!ctx) return fail(PBFTV_EINVAL, "ctx is null");
  if (!ptr) return PBFTV_OK;
  std::vector<void*> evict;
  {
    std::lock_guard<std::mutex> lk(ctx->host_mu);
    auto it = ctx->host_live.find(ptr);
    if (it != ctx->host_live.end()) {
      // kept for the next pbftv_host_alloc: no hipHostFree, so no GPU-wide
      // wait and no halt of the armed servers
      ctx->host_cache.emplace(it->second, ptr);
      ctx->host_cache_bytes += it->second;
      ctx->host_live.erase(it);
      ptr = nullptr;
      while (ctx->host_cache_bytes > pbftv_ctx::kHostCacheBytes) {  // the largest blocks go
        auto big = std::prev(ctx->host_cache.end());
        ctx->host_cache_bytes -= big->first;
        evict.push_back(big->second);
        ctx->host_cache.erase(big);
      }
    }
  }
  if (ptr) evict.push_back(ptr);  // (not ours: freed as before)
  if (!evict.empty()) {
    GpuQuiesce quiet(-1);  // hipHostFree waits for every kernel: armed ones leave first
    for (void* p : evict) HIP_TRY(hipHostFree(p));
  }
  return PBFTV_OK;
}

int pbftv_dev_free(pbftv_ctx* ctx, int dev, void* ptr) {
  Device* d = dev_of(ctx, dev);
  if (!d) return fail(PBFTV_EINVAL, "bad context or device index");
  if (!ptr) return PBFTV_OK;
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  auto it = d->pool_ptrs.find(ptr);
  if (it != d->pool_ptrs.end()) {
    // the block returns to the pool once the context's work queued so far
    // has passed (defer_free / reap_frees)
    d->pool_ptrs.erase(it);
    HIP_TRY(defer_free(*d, ptr));
    HIP_TRY(reap_frees(*d));
    return PBFTV_OK;
  }
  GpuQuiesce quiet(d->id);  // (not from the pool) hipFree waits for every kernel on the GPU: armed ones leave first
  HIP_TRY(hipFree(ptr));
  return PBFTV_OK;
}

int pbftv_memcpy_h2d(pbftv_ctx* ctx, int dev, void* dst, const void* src, uint64_t bytes) {
  Device* d = dev_of(ctx, dev);
  if (!d || (bytes && (!dst || !src))) return fail(PBFTV_EINVAL, "bad argument");
  HIP_TRY(hipSetDevice(d->id));
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, d->stream));
  HIP_TRY(hipStreamSynchronize(d->stream));
  return PBFTV_OK;
}

int pbftv_memcpy_d2h(pbftv_ctx* ctx, int dev, void* dst, const void* src, uint64_t bytes) {
  Device* d = dev_of(ctx, dev);
  if (!d || (bytes && (!dst || !src))) return fail(PBFTV_EINVAL, "bad argument");
  HIP_TRY(hipSetDevice(d->id));
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, d->stream));
  HIP_TRY(hipStreamSynchronize(d->stream));
  return PBFTV_OK;
}

int pbftv_memset_dev(pbftv_ctx* ctx, int dev, void* dst, int value, uint64_t bytes) {
  Device* d = dev_of(ctx, dev);
  if (!d || (bytes && !dst)) return fail(PBFTV_EINVAL, "bad argument");
  HIP_TRY(hipSetDevice(d->id));
  HIP_TRY(hipMemsetAsync(dst, value, bytes, d->stream));
  HIP_TRY(hipStreamSynchronize(d->stream));
  return PBFTV_OK;
}

void* pbftv_stream(pbftv_ctx* ctx, int dev) {
  Device* d = dev_of(ctx, dev);
  return d ? reinterpret_cast<void*>(d->stream) : nullptr;
}

int pbftv_stream_create(pbftv_ctx* ctx, int dev, void** out_stream) {
  Device* d = dev_of(ctx, dev);
  if (!d || !out_stream) return fail(PBFTV_EINVAL, "bad context, device index or out pointer");
  HIP_TRY(hipSetDevice(d->id));
  hipStream_t st;
  HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  {
    std::lock_guard<std::mutex> lk(d->mu);
    d->stream_scratch[st] = std::make_unique<VerifyScratch>();
  }
  *out_stream = reinterpret_cast<void*>(st);
  return PBFTV_OK;
}

int pbftv_stream_destroy(pbftv_ctx* ctx, int dev, void* stream) {
  Device* d = dev_of(ctx, dev);
  if (!d || !stream) return fail(PBFTV_EINVAL, "bad context, device index or stream");
  HIP_TRY(hipSetDevice(d->id));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_TRY(hipStreamSynchronize(st));
  {
    std::lock_guard<std::mutex> lk(d->mu);
    auto it = d->stream_scratch.find(st);
    if (it != d->stream_scratch.end()) {
      it->second->release();
      d->stream_scratch.erase(it);
    }
  }
  HIP_TRY(hipStreamDestroy(st));
  return PBFTV_OK;
}

int pbftv_stream_wait(pbftv_ctx* ctx, int dev, void* stream) {
  Device* d = dev_of(ctx, dev);
  if (!d || !stream) return fail(PBFTV_EINVAL, "bad context, device index or stream");
  HIP_TRY(hipSetDevice(d->id));
  HIP_TRY(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
  return PBFTV_OK;
}

int pbftv_stream_sync(pbftv_ctx* ctx, int dev) {
  Device* d = dev_of(ctx, dev);
  if (!d) return fail(PBFTV_EINVAL, "bad context or device index");
  HIP_TRY(hipSetDevice(d->id));
  HIP_TRY(hipStreamSynchronize(d->stream));
  return PBFTV_OK;
}

int pbftv_set_latency_path_max(pbftv_ctx* ctx, uint64_t n) {
  if (!ctx) return fail(PBFTV_EINVAL, "ctx is null");
  ctx->wave_max.store(n, std::memory_order_relaxed);
  return PBFTV_OK;
}

int pbftv_set_kernel_timing(pbftv_ctx* ctx, int enable) {
  if (!ctx) return fail(PBFTV_EINVAL, "ctx is null");
  ctx->timing = enable != 0;
  return PBFTV_OK;
}

int pbftv_kernel_time_ms(pbftv_ctx* ctx, int dev, int kernel, double* out_ms, uint64_t* out_launches) {
  Device* d = dev_of(ctx, dev);
  if (!d || kernel < 0 || kernel >= Device::kKernels) return fail(PBFTV_EINVAL, "bad argument");
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_TRY(hipSetDevice(d->id));
  HIP_TRY(collect_times(*d));
  if (out_ms) *out_ms = d->acc_ms[kernel];
  if (out_launches) *out_launches = d->launches[kernel];
  return PBFTV_OK;
}

int pbftv_reset_kernel_times(pbftv_ctx* ctx) {
  if (!ctx) return fail(PBFTV_EINVAL, "ctx is null");
  for (auto& dp : ctx->devs) {
    std::lock_guard<std::mutex> lk(dp->mu);
    HIP_TRY(hipSetDevice(dp->id));
    HIP_TRY(collect_times(*dp));
    for (int k = 0; k < Device::kKernels; ++k) {
      dp->acc_ms[k] = 0;
      dp->launches[k] = 0;
    }
  }
  return PBFTV_OK;
}

// ---------------------------------------------------------------- keys
// Comb geometry codes (p256_algo.h CombGeom): W-bit windows, or the mixed
// 21 (5 x 22 + 7 x 21 bits) and 29 (5 x 29 + 4 x 28).  PBFTV_GBITS /
// PBFTV_QBITS force one.
static int env_bits(const char* name, int dflt) {
  const char* e = getenv(name);
  if (!e) return dflt;
  const int v = atoi(e);
  return (v == 8 || v == 12 || v == 16 || v == 20 || v == 21 || v == 22 || v == 24 || v == 26 || v == 29) ? v : dflt;
}

// (G, keys) pairs with instantiated kernels
static bool combo_ok(int wg, int wq) {
#define PBFTV_PAIR(G, Q) \
  if (wg == G && wq == Q) return true;
  PBFTV_COMBOS(PBFTV_PAIR)
#undef PBFTV_PAIR
  return false;
}

// HBM kept free for batch buffers, table-build scratch (~2 GB for 100 keys)
// and other users of the device.
constexpr size_t kTableReserve = 16ull << 30;

// Table geometry: the pair (G, keys) with the fewest windows in total (= mixed
// additions per verify) whose tables fit the device's free HBM minus
// kTableReserve.  An MI355X has 288 GB: G at 29 (mixed) = 120 GB, at 26 =
// 21.5 GB; a key at 24 = 5.9 GB, at 21 (mixed) = 1.14 GB; so 4 keys run
// 9 + 11 windows (144 GB), 100 keys 9 + 12 (234 GB), 1000 keys at 16-bit
// 9 + 17.  Among equal totals the narrower G wins, and for each G the key
// width with the fewest windows, then the least HBM (21 before 22: both 12
// windows).  PBFTV_TABLE_BUDGET_MB caps the key tables.
static void choose_bits(uint32_t k, size_t free_bytes, int* wg, int* wq, const std::function<bool(int)>& g_shared) {
  const uint64_t kk = k ? k : 1;
  const char* env_budget = getenv("PBFTV_TABLE_BUDGET_MB");
  const int force_g = env_bits("PBFTV_GBITS", 0), force_q = env_bits("PBFTV_QBITS", 0);
  int best_g = 0, best_q = 0, best_win = 1 << 30;
  for (int g : {16, 20, 24, 26, 29}) {
    if (force_g && g != force_g) continue;
    const size_t gb = g_shared(g) ? 0 : pbftv::table_bytes(g);  // a G table another context built is free
    size_t budget = free_bytes > kTableReserve + gb ? free_bytes - kTableReserve - gb : 0;
    if (g > 16 && budget == 0 && !force_g) continue;  // wide G tables only with room to spare
    if (g <= 26) budget = std::max(budget, free_bytes / 8);
    if (env_budget) budget = (size_t)atoll(env_budget) << 20;
    for (int q : {24, 21, 22, 20, 16, 12, 8}) {
      if (force_q && q != force_q) continue;
      if (q == 22 && !force_q) continue;  // same windows as 21, 40 % more HBM
      if (!combo_ok(g, q)) continue;
      if (!force_q && q > 8 && kk * pbftv::table_bytes(q) > budget) continue;
      const int win = pbftv::table_windows(g) + pbftv::table_windows(q);
      if (win < best_win) {
        best_win = win;
        best_g = g;
        best_q = q;
      }
      break;  // widest fitting key width for this G
    }
  }
  if (!best_g) {  // forced pair without an instantiated kernel: nearest G for the key width
    best_q = force_q ? force_q : 8;
    best_g = 16;
    for (int g : {force_g, 24, 26, 16, 29})
      if (g && combo_ok(g, best_q)) {
        best_g = g;
        break;
      }
  }
  *wg = best_g;
  *wq = best_q;
}

// PBFTV_TRACE=1: phase timings of key registration on stderr (diagnostics)
static void trace(const char* what, int dev, std::chrono::steady_clock::time_point& t0) {
  static const bool on = getenv("PBFTV_TRACE") != nullptr;
  const auto t1 = std::chrono::steady_clock::now();
  if (on) fprintf(stderr, "pbftv[dev %d] %s: %.1f ms\n", dev, what, std::chrono::duration<double, std::milli>(t1 - t0).count());
  t0 = t1;
}

// Build nb tables of width w (G first when with_g) at the addresses tabs[0..nb)
// (host vector, uploaded here); keys_le: this launch's keys as LE words on the
// device; valid[key0 + j] written for key j of the launch.
static int build_tables(Device& d, int w, const uint32_t* d_keys, uint32_t key0, uint32_t nb, int with_g,
                        uint32_t* valid, const std::vector<void*>& tabs) {
  auto t0 = std::chrono::steady_clock::now();
  const pbftv::TableScratchSizes z = pbftv::table_scratch_sizes(w, nb);
  // grow-only scratch kept by the device: a freed multi-GB buffer is wiped by
  // the driver before its HBM can be handed out again, which costs more than
  // the build
  DevBuf* t = d.tab_scratch;
  HIP_TRY(t[0].ensure(z.bases));
  HIP_TRY(t[1].ensure(z.lbuf));
  HIP_TRY(t[2].ensure(z.hbuf));
  HIP_TRY(t[3].ensure(z.small_scratch));
  HIP_TRY(t[4].ensure(z.entry_scratch));
  HIP_TRY(t[5].ensure(tabs.size() * sizeof(void*)));
  HIP_TRY(hipMemcpyAsync(t[5].p, tabs.data(), tabs.size() * sizeof(void*), hipMemcpyHostToDevice, d.stream));
  trace("table scratch", d.id, t0);
  pbftv::TableScratch sc{t[0].p, t[1].p, t[2].p, t[3].p, t[4].p, z.entry_lanes};
  HIP_TRY(pbftv::launch_build_tables(w, d_keys, key0, nb, with_g, valid, t[5].as<uint32_t* const>(), sc, d.stream));
  HIP_TRY(hipStreamSynchronize(d.stream));
  trace("table kernels", d.id, t0);
  return PBFTV_OK;
}

// big-endian X||Y (64 B per key) -> little-endian 32-bit words {x[8], y[8]}
static std::vector<uint32_t> keys_to_le(const uint8_t* pub_xy, uint32_t k) {
  std::vector<uint32_t> le((size_t)k * 16 + 16);
  for (uint32_t j = 0; j < k; ++j) {
    for (int c = 0; c < 2; ++c) {
      const uint8_t* b = pub_xy + 64ull * j + 32 * c;
      for (int w = 0; w < 8; ++w) {
        const uint8_t* q = b + 4 * (7 - w);
        le[16ull * j + 8 * c + w] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
      }
    }
  }
  return le;
}

// (Re)build the key tables [key0, key0 + k) of d at width d.qbits from host LE
// words, allocating a table for every index past the current ones; refresh the
// device pointer array.  valid_out (host, k entries) gets the key check.
static int build_key_tables(Device& d, const std::vector<uint32_t>& le, uint32_t key0, uint32_t k,
                            uint32_t* valid_out) {
  auto t0 = std::chrono::steady_clock::now();
  const uint32_t total = std::max<uint32_t>(d.nkeys, key0 + k);
  if (d.qtab.size() < total) {  // one block for every table still missing
    const size_t tb = pbftv::table_bytes(d.qbits), more = total - d.qtab.size();
    d.qblocks.push_back(std::make_unique<DevBuf>());
    HIP_TRY(d.qblocks.back()->ensure(more * tb));
    for (size_t j = 0; j < more; ++j) d.qtab.push_back(d.qblocks.back()->as<uint8_t>() + j * tb);
  }
  trace("key table allocation", d.id, t0);
  // key_valid grows with the key count (old flags kept)
  if (d.key_valid.cap < (size_t)total * 4) {
    DevBuf nv;
    HIP_TRY(nv.ensure((size_t)total * 4));
    if (key0 > 0) HIP_TRY(hipMemcpyAsync(nv.p, d.key_valid.p, (size_t)key0 * 4, hipMemcpyDeviceToDevice, d.stream));
    HIP_TRY(hipStreamSynchronize(d.stream));
    std::swap(d.key_valid.p, nv.p);
    std::swap(d.key_valid.cap, nv.cap);
  }
  std::vector<void*> tabs(k);
  for (uint32_t j = 0; j < k; ++j) tabs[j] = d.qtab[key0 + j];
  // the keys' coordinates: a grow-only buffer of the device (a temporary's
  // free would quiesce the GPU -- halt every armed server on it -- at every
  // pbftv_set_key / pbftv_add_keys)
  HIP_TRY(d.tab_keys.ensure((size_t)k * 64 + 64));
  HIP_TRY(hipMemcpyAsync(d.tab_keys.p, le.data(), (size_t)k * 64, hipMemcpyHostToDevice, d.stream));
  if (k) {
    int rc = build_tables(d, d.qbits, d.tab_keys.as<uint32_t>(), key0, k, 0, d.key_valid.as<uint32_t>(), tabs);
    if (rc != PBFTV_OK) return rc;
  }
  trace("key table build", d.id, t0);
  std::vector<void*> ptrs(total);
  for (uint32_t j = 0; j < total; ++j) ptrs[j] = d.qtab[j];
  HIP_TRY(d.qptrs.ensure((size_t)std::max<uint32_t>(total, 1) * sizeof(void*)));
  if (total)
    HIP_TRY(hipMemcpyAsync(d.qptrs.p, ptrs.data(), total * sizeof(void*), hipMemcpyHostToDevice, d.stream));
  if (valid_out && k)
    HIP_TRY(hipMemcpyAsync(valid_out, d.key_valid.as<uint32_t>() + key0, (size_t)k * 4, hipMemcpyDeviceToHost,
                           d.stream));
  HIP_TRY(hipStreamSynchronize(d.stream));
  d.nkeys = total;
  return PBFTV_OK;
}

extern "C++" {
// fn(device) on every device of the context: one host thread per device when
// they are distinct GPUs (the table builds of a registration run in
// parallel), in turn when logical devices share a GPU (PBFTV_ALIAS_DEVICES).
template <class Fn>
static int for_each_device(pbftv_ctx* ctx, Fn fn) {
  bool shared = false;
  for (size_t a = 0; a < ctx->devs.size(); ++a)
    for (size_t b = a + 1; b < ctx->devs.size(); ++b) shared |= ctx->devs[a]->id == ctx->devs[b]->id;
  if (ctx->devs.size() == 1 || shared) {
    for (auto& dp : ctx->devs) {
      int rc = fn(*dp, dp.get() == ctx->devs[0].get());
      if (rc != PBFTV_OK) return rc;
    }
    return PBFTV_OK;
  }
  std::vector<int> rc(ctx->devs.size(), PBFTV_OK);
  std::vector<std::string> errs(ctx->devs.size());
  std::vector<std::thread> th;
  for (size_t i = 0; i < ctx->devs.size(); ++i)
    th.emplace_back([&, i] {
      rc[i] = fn(*ctx->devs[i], i == 0);
      if (rc[i] != PBFTV_OK) errs[i] = g_last_error;
    });
  for (auto& t : th) t.join();
  for (size_t i = 0; i < rc.size(); ++i)
    if (rc[i] != PBFTV_OK) return fail(rc[i], errs[i]);
  return PBFTV_OK;
}
}  // extern "C++"

// One attempt at a device's tables: geometry from the HBM free now, then the G
// table (shared per GPU and width) and the key tables (pbftv_register_keys).
static int register_tables(Device& d, const std::vector<uint32_t>& le, uint32_t k, uint32_t* valid,
                           std::chrono::steady_clock::time_point t0) {
  size_t free_b = 0, total_b = 0, held = 0;
  HIP_TRY(hipMemGetInfo(&free_b, &total_b));
  for (auto& b : d.qblocks) held += b->cap;  // the old key tables' HBM counts for the new ones
  int wg, wq;
  const int dev_id = d.id;
  choose_bits(k, free_b + held, &wg, &wq, [&](int g) {
    std::lock_guard<std::mutex> gl(g_tables_mu);
    auto it = g_tables.find({dev_id, g});
    return it != g_tables.end() && !it->second.tab.expired();  // ours or another context's: no new HBM
  });
  trace("geometry", d.id, t0);
  d.nkeys = 0;
  if (wq != d.qbits || d.qtab.size() < k) {  // new width or too few slots: new blocks (freeing HBM
    for (auto& b : d.qblocks) b->release();  // the driver wipes is slow: same-width re-registrations
    d.qblocks.clear();                       // reuse their slots)
    d.qtab.clear();
  }
  trace("release old key tables", d.id, t0);
  if (d.gbits != wg || !d.gtab) {  // G table: once per GPU and width while any context holds it
    d.gtab.reset();
    d.gbits = 0;
    std::shared_ptr<std::mutex> build_mu;
    {
      std::lock_guard<std::mutex> gl(g_tables_mu);
      build_mu = g_tables[{d.id, wg}].build;
    }
    std::lock_guard<std::mutex> bl(*build_mu);  // one builder per (GPU, width); others wait here, not globally
    {
      std::lock_guard<std::mutex> gl(g_tables_mu);
      d.gtab = g_tables[{d.id, wg}].tab.lock();
    }
    if (!d.gtab) {
      auto t = std::make_shared<DevBuf>();
      HIP_TRY(t->ensure(pbftv::table_bytes(wg)));
      DevBuf dummy;
      HIP_TRY(dummy.ensure(64));
      trace("G table allocation", d.id, t0);
      const int r = build_tables(d, wg, nullptr, 0, 1, 1, dummy.as<uint32_t>(), {t->p});
      if (r != PBFTV_OK) return r;
      trace("G table build", d.id, t0);
      {
        std::lock_guard<std::mutex> gl(g_tables_mu);
        g_tables[{d.id, wg}].tab = t;
      }
      d.gtab = std::move(t);
    }
    d.gbits = wg;
  }
  d.qbits = wq;
  const int r = build_key_tables(d, le, 0, k, valid);
  if (r != PBFTV_OK) return r;
  d.have_keys = true;
  return PBFTV_OK;
}

int pbftv_register_keys(pbftv_ctx* ctx, const uint8_t* pub_xy, uint32_t k, uint8_t* out_valid) {
  if (!ctx || (k && !pub_xy)) return fail(PBFTV_EINVAL, "null argument");
  const std::vector<uint32_t> le = keys_to_le(pub_xy, k);
  std::vector<uint32_t> valid(k ? k : 1, 0);
  int rc = for_each_device(ctx, [&](Device& d, bool first) -> int {
    std::lock_guard<std::mutex> lk(d.mu);
    HIP_TRY(hipSetDevice(d.id));
    auto t0 = std::chrono::steady_clock::now();
    // nothing of this context still reads the tables, key_valid or qptrs this
    // call rewrites in place: its armed kernels, its streams and the caller
    // streams it was given (a verify enqueued on one with *_dev)
    HIP_TRY(ctx_quiesce(d));
    trace("quiesce", d.id, t0);
    d.have_keys = false;
    // another process or context can take HBM between the free-memory query
    // and the allocations: on ENOMEM this device's tables are freed and the
    // geometry is chosen again from what is free then (3 attempts)
    for (int attempt = 0;; ++attempt) {
      const int r = register_tables(d, le, k, first ? valid.data() : nullptr, t0);
      if (r != PBFTV_ENOMEM || attempt == 2) return r;
      for (auto& b : d.qblocks) b->release();
      d.qblocks.clear();
      d.qtab.clear();
      d.gtab.reset();
      d.gbits = d.qbits = 0;
      d.nkeys = 0;
    }
  });
  if (rc != PBFTV_OK) {
    for (auto& dp : ctx->devs) {  // no device keeps a key set the others lack
      std::lock_guard<std::mutex> lk(dp->mu);
      dp->have_keys = false;
    }
    return rc;
  }
  if (out_valid)
    for (uint32_t j = 0; j < k; ++j) out_valid[j] = valid[j] ? 1 : 0;
  return PBFTV_OK;
}

int pbftv_add_keys(pbftv_ctx* ctx, const uint8_t* pub_xy, uint32_t k, uint8_t* out_valid) {
  if (!ctx || (k && !pub_xy)) return fail(PBFTV_EINVAL, "null argument");
  if (!keys_ready(ctx)) return fail(PBFTV_ENOKEYS, "pbftv_register_keys has not been called");
  const std::vector<uint32_t> le = keys_to_le(pub_xy, k);
  std::vector<uint32_t> valid(k ? k : 1, 0);
  int rc = for_each_device(ctx, [&](Device& d, bool first) -> int {
    std::lock_guard<std::mutex> lk(d.mu);
    HIP_TRY(hipSetDevice(d.id));
    HIP_TRY(ctx_quiesce(d));  // (as in pbftv_register_keys: qptrs and key_valid are rewritten)
    return build_key_tables(d, le, d.nkeys, k, first ? valid.data() : nullptr);
  });
  if (rc != PBFTV_OK) {
    // a device that failed (or succeeded) leaves the key counts disagreeing
    // across shards: every device is unusable until the caller re-registers
    for (auto& dp : ctx->devs) {
      std::lock_guard<std::mutex> lk(dp->mu);
      dp->have_keys = false;
    }
    return rc;
  }
  if (out_valid)
    for (uint32_t j = 0; j < k; ++j) out_valid[j] = valid[j] ? 1 : 0;
  return PBFTV_OK;
}

int pbftv_set_key(pbftv_ctx* ctx, uint32_t index, const uint8_t* pub_xy, uint8_t* out_valid) {
  if (!ctx || !pub_xy) return fail(PBFTV_EINVAL, "null argument");
  if (!keys_ready(ctx)) return fail(PBFTV_ENOKEYS, "pbftv_register_keys has not been called");
  for (auto& dp : ctx->devs)
    if (index >= dp->nkeys) return fail(PBFTV_EINVAL, "key index out of range");
  const std::vector<uint32_t> le = keys_to_le(pub_xy, 1);
  uint32_t valid = 0;
  int rc = for_each_device(ctx, [&](Device& d, bool first) -> int {
    std::lock_guard<std::mutex> lk(d.mu);
    HIP_TRY(hipSetDevice(d.id));
    HIP_TRY(ctx_quiesce(d));  // no verify of this context (caller streams too) still reads the old table
    return build_key_tables(d, le, index, 1, first ? &valid : nullptr);
  });
  if (rc != PBFTV_OK) {
    for (auto& dp : ctx->devs) {  // devices may now disagree on key `index`: re-register first
      std::lock_guard<std::mutex> lk(dp->mu);
      dp->have_keys = false;
    }
    return rc;
  }
  if (out_valid) *out_valid = valid ? 1 : 0;
  return PBFTV_OK;
}

int pbftv_table_config(const pbftv_ctx* ctx, int* out_gbits, int* out_qbits, uint64_t* out_table_bytes) {
  if (!ctx || ctx->devs.empty()) return fail(PBFTV_EINVAL, "ctx is null");
  const Device& d = *ctx->devs[0];
  if (out_gbits) *out_gbits = d.gbits;
  if (out_qbits) *out_qbits = d.qbits;
  if (out_table_bytes)
    *out_table_bytes = (d.gbits ? pbftv::table_bytes(d.gbits) : 0) + (d.qbits ? (uint64_t)d.nkeys * pbftv::table_bytes(d.qbits) : 0);
  return PBFTV_OK;
}

// ---------------------------------------------------------------- ecdsa
// Lane path (or the one-wave-per-signature path for small n) of one batch on
// stream st.  own == nullptr: the device's shared scratch, ordered across
// streams by the scratch event; else the caller's (a pipeline stream's own).
// a lane-path batch of n signatures was enqueued on d: ~ns_per_sig of device
// time per signature (1.1: the device-resident 1M step; the host-buffer path
// is PCIe-bound at ~2.3), queued behind what is already there.  With
// PBFTV_QC_YIELD an armed kernel of d is halted now (it leaves at its next
// poll; a certificate meanwhile takes a launch) -- d.mu is held.
static void note_busy(Device& d, uint64_t n, double ns_per_sig = 1.1) {
  const int64_t now = steady_ns(), add = (int64_t)(ns_per_sig * (double)n) + 20000;
  int64_t cur = d.busy_until_ns.load(std::memory_order_relaxed);
  while (!d.busy_until_ns.compare_exchange_weak(cur, std::max(cur, now) + add, std::memory_order_relaxed)) {
  }
  if (d.arm_seq && qc_yield_now(d) && d.stage.p && d.mail_registered) {
    __atomic_add_fetch(&qc_mail(d)->halt, 1u, __ATOMIC_RELEASE);
    d.arm_seq = 0;
    d.retiring = 0;
  }
}

// the device a latency-path call goes to: devs[0] unless it is busy with
// lane-path batches and another device is less so (an idle device with an
// armed server first, then the earliest-free one)
static Device* latency_device(pbftv_ctx* ctx) {
  Device* best = ctx->dev0;
  if (ctx->devs.size() == 1) return best;
  const int64_t now = steady_ns();
  int64_t best_free = std::max<int64_t>(best->busy_until_ns.load(std::memory_order_relaxed), now);
  if (best_free <= now) return best;
  for (auto& dp : ctx->devs) {
    const int64_t f = std::max<int64_t>(dp->busy_until_ns.load(std::memory_order_relaxed), now);
    if (f < best_free || (f == best_free && f <= now && dp->arm_seq.load(std::memory_order_relaxed) &&
                          !best->arm_seq.load(std::memory_order_relaxed))) {
      best = dp.get();
      best_free = f;
    }
  }
  return best;
}

static int verify_on_device(Device& d, const uint8_t* d_hashes, const uint8_t* d_sigs, const uint32_t* d_key_idx,
                            uint64_t n, uint8_t* d_bitmap, hipStream_t st, VerifyScratch* own = nullptr) {
  if (!d.have_keys) return fail(PBFTV_ENOKEYS, "pbftv_register_keys has not been called");
  if (n <= d.wave_max->load(std::memory_order_relaxed)) {
    HIP_TRY(timed(d, PBFTV_K_ECDSA_WAVE, st, [&] {
      return pbftv::launch_ecdsa_wave(d.gbits, d.qbits, d_hashes, d_sigs, d_key_idx, n, d.key_valid.as<uint32_t>(),
                                      d.nkeys, d.gtab->as<uint32_t>(), d.qptrs.as<const uint32_t* const>(), d_bitmap, nullptr, st);
    }));
    HIP_TRY(fence_reader(d, st));
    return PBFTV_OK;
  }
  if (!own) {
    auto it = d.stream_scratch.find(st);
    if (it != d.stream_scratch.end()) own = it->second.get();
  }
  VerifyScratch& sc = own ? *own : d.vs;
  note_busy(d, n);
  HIP_TRY(sc.rec.ensure(pbftv::ecdsa_record_bytes(n)));
  HIP_TRY(sc.prefix.ensure(pbftv::scalar_prefix_bytes(n)));
  if (!own) HIP_TRY(scratch_acquire(d, st));
  const bool sorted = pbftv::key_sort_wanted(n, d.nkeys);
  pbftv::KeyOrder ko{nullptr, nullptr, 0};
  if (sorted) {
    HIP_TRY(sc.okb.ensure(n));  // comb lanes in key order: a wave's table lookups share keys (p256_kernels.hip k_key_*)
    HIP_TRY(ensure_key_sort(sc, n, d.nkeys, st));
    HIP_TRY(pbftv::launch_key_count(d_key_idx, n, d.nkeys, sc.ksort.p, sc.sort_parity++, &ko, st));
  }
  HIP_TRY(timed(d, PBFTV_K_ECDSA_SCALARS, st, [&] {
    return pbftv::launch_ecdsa_scalars(d_hashes, d_sigs, d_key_idx, n, d.key_valid.as<uint32_t>(), d.nkeys, sc.rec.p,
                                       sc.prefix.p, ko, st);
  }));
  HIP_TRY(timed(d, PBFTV_K_ECDSA_COMB, st, [&] {
    return pbftv::launch_ecdsa_comb(d.gbits, d.qbits, sc.rec.p, n, d.gtab->as<uint32_t>(),
                                    d.qptrs.as<const uint32_t* const>(), d_bitmap,
                                    sorted ? sc.okb.as<uint8_t>() : nullptr,
                                    // (only while a server is armed: the comb's
                                    // per-step read of its CU's word costs ~0.4 %)
                                    qc_cu_yield() && d.arm_seq.load(std::memory_order_relaxed)
                                        ? d.cuflag_ready.load(std::memory_order_acquire)
                                        : nullptr,
                                    st);
  }));
  if (sorted) HIP_TRY(pbftv::launch_pack_bits(sc.okb.as<uint8_t>(), n, d_bitmap, st));
  if (!own) HIP_TRY(scratch_release(d, st));
  return PBFTV_OK;
}

// Host-buffer verify of one shard, pipelined in chunks: the copies of every
// chunk are queued back to back on one copy stream (each into its own device
// slot, up to PBFTV_HOST_SLOTS = 16 ahead, so the PCIe link never waits for
// a slot to be verified), and chunk k is verified as soon as its copy has
// landed: even chunks on d.stream, odd chunks on d.stream2 with their own
// scratch (so two chunks' verifies can overlap at the end of the batch).  The caller's buffers are DMA'd as they are: pinned memory
// directly, pageable memory through the runtime's own staging (faster than a
// parallel memcpy into pinned slots, profiles/r02_ab_host_path.jsonl).  The
// bitmap comes back in one copy at the end.  Chunk sizes are multiples of 512
// (bitmap bytes and waves stay aligned).
static bool env_flag(const char* name, bool dflt) {
  const char* e = getenv(name);
  return e ? e[0] == '1' : dflt;
}

static uint64_t host_chunk() {
  uint64_t c = 262144;
  if (const char* e = getenv("PBFTV_HOST_CHUNK")) c = std::max<uint64_t>(512, strtoull(e, nullptr, 10));
  return (c + 511) / 512 * 512;
}

// Chunk sizes for m items: whole chunks, then a short last chunk (default
// 131072, PBFTV_HOST_LAST), since the last chunk's verify is the one part no
// copy hides.  (Halving every chunk of the tail measured slower: each DMA
// command costs a ~10-20 us gap on the copy engine; tools/host_path_ab.py.)
static std::vector<uint64_t> host_chunks(uint64_t m) {
  const uint64_t c = host_chunk();
  uint64_t last = 131072;  // (65536 / 32768 measured slower with the second verify stream)
  if (const char* e = getenv("PBFTV_HOST_LAST")) last = strtoull(e, nullptr, 10) / 512 * 512;
  if (last >= c || m <= c) last = 0;
  // every chunk but the final one is a multiple of 512 (each chunk's bitmap
  // starts on a byte): the ragged remainder joins the last chunk
  const uint64_t head = last ? (m - last) / 512 * 512 : m;
  std::vector<uint64_t> out;
  for (uint64_t r = head; r > 0; r -= std::min(c, r)) out.push_back(std::min(c, r));
  if (m > head) out.push_back(m - head);
  return out;
}

static int host_slots() {
  int s = Device::kSlots;
  if (const char* e = getenv("PBFTV_HOST_SLOTS")) s = atoi(e);
  return std::min(Device::kSlots, std::max(2, s));
}

static int verify_host_pipelined(Device& d, const uint8_t* H, const uint8_t* S, const uint32_t* K, uint64_t m,
                                 uint8_t* out_bm) {
  const std::vector<uint64_t> chunks = host_chunks(m);
  const uint64_t c = *std::max_element(chunks.begin(), chunks.end()), nch = chunks.size();
  note_busy(d, m, 1.2);  // the PCIe-bound part beyond the chunks' own verify time (~2.3 ns per signature in all)
  const int ns = (int)std::min<uint64_t>(nch, host_slots());
  const size_t oh = 0, os = 32 * c, ok = 96 * c, slot = 100 * c;  // slot layout: hashes | sigs | keys
  // every key index in one copy up front (one DMA command per chunk fewer;
  // PBFTV_HOST_KEYS_FIRST=0 disables), and odd chunks verified on a second
  // stream with their own scratch, so the last chunks' verifies overlap instead
  // of queueing behind each other (PBFTV_HOST_2COMPUTE=0 disables).  Same box:
  // pinned 2.38 -> 2.30 ms, pageable 2.46 -> 2.36 ms (profiles/r02_ab_host_path_2compute.jsonl;
  // a second copy queue for the signatures measured no gain).
  const bool keys_first = env_flag("PBFTV_HOST_KEYS_FIRST", true);
  const bool two = env_flag("PBFTV_HOST_2COMPUTE", true) && nch > 1;
  if (two) {
    if (!d.stream2) HIP_TRY(hipStreamCreateWithFlags(&d.stream2, hipStreamNonBlocking));
    if (!d.join_ev) HIP_TRY(hipEventCreateWithFlags(&d.join_ev, hipEventDisableTiming));
  }
  if (!d.cstream) HIP_TRY(hipStreamCreateWithFlags(&d.cstream, hipStreamNonBlocking));
  for (int k = 0; k < ns; ++k) {
    if (!d.h2d_ev[k]) HIP_TRY(hipEventCreateWithFlags(&d.h2d_ev[k], hipEventDisableTiming));
    if (!d.comp_ev[k]) HIP_TRY(hipEventCreateWithFlags(&d.comp_ev[k], hipEventDisableTiming));
    HIP_TRY(d.din[k].ensure(slot + 64));
  }
  HIP_TRY(d.bitmap.ensure((m + 7) / 8 + 8));
  if (keys_first) {
    HIP_TRY(d.keys_all.ensure(4 * m + 64));
    HIP_TRY(hipMemcpyAsync(d.keys_all.p, K, 4 * m, hipMemcpyHostToDevice, d.cstream));
  }
  bool used[Device::kSlots] = {};
  uint64_t lo = 0;
  for (uint64_t j = 0; j < nch; lo += chunks[j], ++j) {
    const int k = (int)(j % ns);
    const uint64_t cnt = chunks[j];
    uint8_t* dv = d.din[k].as<uint8_t>();
    if (used[k]) HIP_TRY(hipStreamWaitEvent(d.cstream, d.comp_ev[k], 0));  // slot's previous chunk verified
    HIP_TRY(hipMemcpyAsync(dv + oh, H + 32 * lo, 32 * cnt, hipMemcpyHostToDevice, d.cstream));
    HIP_TRY(hipMemcpyAsync(dv + os, S + 64 * lo, 64 * cnt, hipMemcpyHostToDevice, d.cstream));
    if (!keys_first) HIP_TRY(hipMemcpyAsync(dv + ok, K + lo, 4 * cnt, hipMemcpyHostToDevice, d.cstream));
    hipStream_t vst = two && (j & 1) ? d.stream2 : d.stream;
    HIP_TRY(hipEventRecord(d.h2d_ev[k], d.cstream));
    HIP_TRY(hipStreamWaitEvent(vst, d.h2d_ev[k], 0));
    const uint32_t* kp = keys_first ? d.keys_all.as<uint32_t>() + lo : reinterpret_cast<const uint32_t*>(dv + ok);
    int rc = verify_on_device(d, dv + oh, dv + os, kp, cnt, d.bitmap.as<uint8_t>() + lo / 8, vst,
                              vst == d.stream2 ? &d.vs2 : nullptr);
    if (rc != PBFTV_OK) return rc;
    HIP_TRY(hipEventRecord(d.comp_ev[k], vst));
    used[k] = true;
  }
  if (two) {  // the bitmap copy waits for both verify streams
    HIP_TRY(hipEventRecord(d.join_ev, d.stream2));
    HIP_TRY(hipStreamWaitEvent(d.stream, d.join_ev, 0));
  }
  HIP_TRY(hipMemcpyAsync(out_bm, d.bitmap.p, (m + 7) / 8, hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(hipStreamSynchronize(d.stream));
  return PBFTV_OK;
}

int pbftv_ecdsa_p256_verify_batch_dev(pbftv_ctx* ctx, int dev, const uint8_t* d_hashes, const uint8_t* d_sig_rs,
                                      const uint32_t* d_key_idx, uint64_t n, uint8_t* d_bitmap, void* stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return fail(PBFTV_EINVAL, "bad context or device index");
  if (n && (!d_hashes || !d_sig_rs || !d_key_idx || !d_bitmap)) return fail(PBFTV_EINVAL, "null buffer");
  if (((uintptr_t)d_hashes | (uintptr_t)d_sig_rs) & 15u) return fail(PBFTV_EINVAL, "hashes/sigs must be 16-B aligned");
  Device& d = *ctx->devs[dev];
  std::lock_guard<std::mutex> lk(d.mu);
  HIP_TRY(hipSetDevice(d.id));
  return verify_on_device(d, d_hashes, d_sig_rs, d_key_idx, n, d_bitmap, pick_stream(d, stream));
}

int pbftv_ecdsa_p256_verify_batch(pbftv_ctx* ctx, const uint8_t* hashes, const uint8_t* sig_rs,
                                  const uint32_t* key_idx, uint64_t n, uint8_t* out_bitmap) {
  const auto h_entry = std::chrono::steady_clock::now();
  if (!ctx) return fail(PBFTV_EINVAL, "ctx is null");
  if (n && (!hashes || !sig_rs || !key_idx || !out_bitmap)) return fail(PBFTV_EINVAL, "null buffer");
  Device* const ldev = n && ctx->dev0 ? latency_device(ctx) : nullptr;
  if (n && n <= QcMail::kQcCap && ldev) {
    // A certificate after an idle second finds this core's caches cold (the
    // caller slept; its core's private caches were flushed): start the misses
    // of the lines the armed path touches now, in parallel, instead of one
    // after another (device lock and state, the mailbox header, slot lines and
    // verdict bytes: the mailbox's first page).  A stale mailbox pointer is
    // harmless: a prefetch never faults.
    const Device* d0 = ldev;
    for (const char* q = reinterpret_cast<const char*>(&d0->mu); q <= d0->hot_end; q += 64) __builtin_prefetch(q, 1, 3);
    __builtin_prefetch(d0->hot_end, 1, 3);
    if (const uint8_t* mb = static_cast<const uint8_t*>(d0->stage.p)) {
      for (size_t off = 0; off < QcMail::arrays_off(); off += 64) __builtin_prefetch(mb + off, 1, 3);
      if (n > QcMail::kQcSlots) {  // the helpers' input arrays this call writes
        const uint64_t h = n - QcMail::kQcSlots;
        for (uint64_t off = 0; off < 32 * h; off += 64)
          __builtin_prefetch(mb + QcMail::hashes_off() + 32 * QcMail::kQcSlots + off, 1, 3);
        for (uint64_t off = 0; off < 64 * h; off += 64)
          __builtin_prefetch(mb + QcMail::sigs_off(QcMail::kQcCap) + 64 * QcMail::kQcSlots + off, 1, 3);
        for (uint64_t off = 0; off < 4 * h; off += 64)
          __builtin_prefetch(mb + QcMail::keys_off(QcMail::kQcCap) + 4 * QcMail::kQcSlots + off, 1, 3);
      }
    }
    // and the caller's buffers
    for (uint64_t off = 0; off < 32 * n; off += 64) __builtin_prefetch(hashes + off, 0, 3);
    for (uint64_t off = 0; off < 64 * n; off += 64) __builtin_prefetch(sig_rs + off, 0, 3);
    for (uint64_t off = 0; off < 4 * n; off += 64) __builtin_prefetch(key_idx + off / 4, 0, 3);
    __builtin_prefetch(out_bitmap, 1, 3);
  }
  for (auto& dp : ctx->devs)
    if (!dp->have_keys) return fail(PBFTV_ENOKEYS, "pbftv_register_keys has not been called");
  if (n && n <= ctx->wave_max.load(std::memory_order_relaxed)) {
    // latency path on the first device: inputs packed into pinned coherent
    // host memory (the QcMail mailbox) that the kernel reads directly, one byte
    // per signature written back the same way and polled for (sentinel 0xFF):
    // no copies, no stream synchronisation on the fast path.  Up to kQcSlots
    // signatures (a certificate of n <= 9 replicas) are served by the ARMED
    // kernel (k_ecdsa_wave_armed), a persistent server kept waiting on this
    // device (qc_arm, qc_keeper_loop): the request writes its slot lines and
    // rings, and nothing else -- no launch, no HIP call -- is on its path.
    // Otherwise, or when the armed kernel has run out, one launch of
    // k_ecdsa_wave (up to 2048 signatures, one wave each).  In a multi-device
    // context the call goes to the least-loaded device (latency_device).
    Device& d = *ldev;
    std::lock_guard<std::mutex> lk(d.mu);
    const auto h_in = std::chrono::steady_clock::now();
    d.last_qc = h_in;
    bool dev_set = false;
    auto set_dev = [&]() -> hipError_t {  // only paths that make HIP calls pay for it
      if (dev_set) return hipSuccess;
      dev_set = true;
      return hipSetDevice(d.id);
    };
    const bool small = n <= kQcCap;
    const uint32_t cap = small ? kQcCap : (uint32_t)n;  // the armed kernels assume kQcCap (QcMail::kQcCap)
    if (!small || d.stage.cap < QcMail::bytes(cap) || !d.mail_registered) {
      HIP_TRY(set_dev());
      HIP_TRY(qc_disarm(d));  // (the mailbox is relaid out for n)
      HIP_TRY(qc_mail_layout(d, cap));
    }
    QcMail* m = qc_mail(d);
    uint8_t* st8 = d.stage.as<uint8_t>();
    volatile uint8_t* const res = st8 + QcMail::res_off(cap);
    std::memset(const_cast<uint8_t*>(res), 0xFF, n);
    m->cap = cap;
    m->n = (uint32_t)n;
    ++d.qc_calls;
    hipStream_t lst = nullptr;  // where this call's launched kernel went (latency_stream)
    // one launch of the latency kernel for signatures [lo, n), inputs from
    // the mailbox arrays, result bytes in place
    auto launch_range = [&](uint64_t lo) -> int {
      ++d.qc_launches;
      uint8_t* const hp = st8 + QcMail::hashes_off(cap) + 32 * lo;
      uint8_t* const sp = st8 + QcMail::sigs_off(cap) + 64 * lo;
      uint32_t* const kp = reinterpret_cast<uint32_t*>(st8 + QcMail::keys_off(cap)) + lo;
      std::memcpy(hp, hashes + 32 * lo, 32 * (n - lo));
      std::memcpy(sp, sig_rs + 64 * lo, 64 * (n - lo));
      std::memcpy(kp, key_idx + lo, 4 * (n - lo));
      HIP_TRY(set_dev());
      HIP_TRY(latency_stream(d, &lst));
      // beside this device's lane batches: one wave per signature (a row
      // workgroup would wait for several freed wave slots on one CU)
      // (PBFTV_QC_BUSY_ONE_WAVE=0: never; =2: always -- tests of the one-wave kernel)
      const char* ow = getenv("PBFTV_QC_BUSY_ONE_WAVE");
      const bool one_wave = ow && ow[0] == '2' ? true : lane_busy(d) && !(ow && ow[0] == '0');
      HIP_TRY(timed(d, PBFTV_K_ECDSA_WAVE, lst, [&] {
        return pbftv::launch_ecdsa_wave(d.gbits, d.qbits, hp, sp, kp, n - lo, d.key_valid.as<uint32_t>(), d.nkeys,
                                        d.gtab->as<uint32_t>(), d.qptrs.as<const uint32_t* const>(), nullptr,
                                        const_cast<uint8_t*>(res) + lo, lst, one_wave);
      }));
      return PBFTV_OK;
    };
    auto launch_plain = [&]() -> int { return launch_range(0); };
    // an armed kernel that has left (budget, cancel, halt) is collected first
    bool collected = false;
    if (d.arm_seq && __atomic_load_n(m->expired(d.arm_stream), __ATOMIC_ACQUIRE) == d.arm_seq) {
      HIP_TRY(set_dev());
      HIP_TRY(qc_disarm(d));
      collected = true;
    }
    const bool trace_qc = trace_qc_enabled();
    if (trace_qc && small && d.arm_seq && n <= d.arm_waves && n > QcMail::kQcSlots && !qc_all_live(d)) {
      const uint32_t* lv = reinterpret_cast<const uint32_t*>(d.stage.as<uint8_t>() + QcMail::live_off(d.arm_stream));
      uint32_t k = 0;
      for (uint32_t w = 0; w < d.arm_waves; ++w) k += __atomic_load_n(lv + w, __ATOMIC_ACQUIRE) == d.armed_first;
      fprintf(stderr, "pbftv[dev %d] qc n=%llu launched: %u of %u workgroups of armed %u live (armed %.1f ms ago, retiring %u)\n",
              d.id, (unsigned long long)n, k, d.arm_waves, d.arm_seq.load(),
              std::chrono::duration<double, std::milli>(h_in - d.armed_at).count(), d.retiring);
    }
    if (trace_qc && small && !(d.arm_seq && n <= d.arm_waves))  // (diagnostics: why a launch)
      fprintf(stderr, "pbftv[dev %d] qc n=%llu launched: arm_seq=%u arm_waves=%u collected=%d wide_wanted=%d retiring=%u\n",
              d.id, (unsigned long long)n, d.arm_seq.load(), d.arm_waves, (int)collected, (int)qc_wide_wanted(d), d.retiring);
    uint32_t cur = 0;  // the armed request number serving this call
    if (n > QcMail::kQcSlots && small) d.last_wide = h_in;
    if (n <= QcMail::kQcSlots) d.qc_nmax = std::max(d.qc_nmax, (uint32_t)n);
    else if (small) d.qc_wmax = std::max(d.qc_wmax, (uint32_t)n);
    // a wide certificate needs every helper workgroup resident: one that is
    // still waiting for room on the GPU (beside other resident kernels) would
    // start only after the armed kernel's budget, too late to serve
    // PBFTV_QC_WIDE=split: a certificate wider than the narrow server is split
    // -- its first signatures go to the armed slots, the rest to one launch
    // beside them (no wide server resident between certificates)
    const bool split = small && n > QcMail::kQcSlots && d.arm_seq && !d.arm_wide && qc_wide_mode() == 2;
    if (d.arm_seq && (split || (n <= d.arm_waves && (n <= QcMail::kQcSlots || qc_all_live(d))))) {
      cur = d.arm_seq;
      const uint64_t na = split ? std::min<uint64_t>(n, d.arm_waves) : n;  // signatures the armed kernel serves
      if (n > QcMail::kQcSlots && !split) {  // the helpers' inputs (slots kQcSlots..n-1), before any slot tag
        std::memcpy(st8 + QcMail::hashes_off(cap) + 32 * QcMail::kQcSlots, hashes + 32 * QcMail::kQcSlots,
                    32 * (n - QcMail::kQcSlots));
        std::memcpy(st8 + QcMail::sigs_off(cap) + 64 * QcMail::kQcSlots, sig_rs + 64 * QcMail::kQcSlots,
                    64 * (n - QcMail::kQcSlots));
        std::memcpy(st8 + QcMail::keys_off(cap) + 4 * QcMail::kQcSlots, key_idx + QcMail::kQcSlots,
                    4 * (n - QcMail::kQcSlots));
      }
      // the kernel waits for cur + 1 next (0 is "none": cancel it at the wrap)
      d.arm_seq = d.seq_counter = cur + 1;
      // the slots: each line's data, then its tags (a line is read by the GPU
      // as one snapshot, and x86 stores become visible in order)
      for (uint32_t i = 0; i < QcMail::kQcSlots; ++i) {
        uint32_t* l0 = reinterpret_cast<uint32_t*>(st8 + QcMail::slot_off(i));
        uint32_t* l1 = l0 + 16;
        uint32_t* l2 = l0 + 32;
        if (i < na) {
          std::memcpy(l0 + 4, hashes + 32 * i, 32);
          std::memcpy(l1 + 4, sig_rs + 64 * i, 32);
          std::memcpy(l2 + 4, sig_rs + 64 * i + 32, 32);
          l0[2] = key_idx[i];
          for (uint32_t* l : {l1, l2}) {
            __atomic_store_n(l + 15, cur, __ATOMIC_RELEASE);
            __atomic_store_n(l, cur, __ATOMIC_RELEASE);
          }
        }
        l0[1] = (uint32_t)na;  // a slot past na: line 0 only (its wave reads na and waits for the next)
        __atomic_store_n(l0 + 15, cur, __ATOMIC_RELEASE);
        __atomic_store_n(l0, cur, __ATOMIC_RELEASE);
      }
      __atomic_store_n(&m->bell, cur, __ATOMIC_RELEASE);  // inputs and n are in: ring
      if (na < n) {  // (split) the rest in one launch, beside the armed slots
        int rc = launch_range(na);
        if (rc != PBFTV_OK) return rc;
      }
    } else {
      // a batch the armed kernel cannot take (n > its waves) leaves it armed
      // for the next small one; a narrow one is replaced by a wide one for the
      // next certificate of this size (qc_wide_wanted)
      int rc = launch_plain();
      if (rc != PBFTV_OK) return rc;
      if (small) {
        // wide, or more slots (qc_nmax / qc_wmax), for the next one -- unless
        // PBFTV_QC_SLOTS fixes the narrow shape, which would re-arm the same
        const bool narrow_fixed = n <= QcMail::kQcSlots && qc_slots_fixed() && !qc_wide_wanted(d);
        if (d.arm_seq && n > d.arm_waves && (qc_wide_wanted(d) || n <= QcMail::kQcSlots) && !narrow_fixed)
          HIP_TRY(qc_rotate(d));
        HIP_TRY(qc_arm(d));  // the next call's server (no-op while one is armed)
      }
    }
    const auto h_bell = std::chrono::steady_clock::now();
    // every wave writes its byte after its last read of the inputs, so once
    // all n bytes are in, the mailbox is free for the next call
    auto t0 = std::chrono::steady_clock::now();
    const uint64_t slots_n = std::min<uint64_t>(n, QcMail::kQcSlots);
    auto h_slots = h_bell;
    for (uint64_t next = 0; next < n;) {
      if (res[next] != 0xFF) {
        if (++next == slots_n) h_slots = std::chrono::steady_clock::now();
        continue;
      }
      if (cur && __atomic_load_n(m->expired(d.arm_stream), __ATOMIC_ACQUIRE) == cur) {
        // the armed kernel left (budget, cancel, halt) before it saw the bell:
        // wait for the armed kernels to leave, then launch
        if (trace_qc)
          fprintf(stderr, "pbftv[dev %d] qc n=%llu: armed %u left unserved after %.1f us (halt %u, stop %u, armed %.1f ms ago)\n",
                  d.id, (unsigned long long)n, cur,
                  std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h_in).count(), m->halt,
                  m->stop, std::chrono::duration<double, std::milli>(h_in - d.armed_at).count());
        HIP_TRY(set_dev());
        HIP_TRY(qc_disarm(d));
        cur = 0;
        std::memset(const_cast<uint8_t*>(res), 0xFF, n);
        int rc = launch_plain();
        if (rc != PBFTV_OK) return rc;
        HIP_TRY(qc_arm(d));
        next = 0;
        t0 = std::chrono::steady_clock::now();
        continue;
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        // nothing that served (or could still serve) this call may outlive the
        // return: the armed kernels and the launched one have left after these
        // synchronisations (a kernel fault surfaces here as a stream error), so
        // no stale verdict can land in the next call's result bytes
        HIP_TRY(set_dev());
        HIP_TRY(qc_disarm(d));
        if (lst) HIP_TRY(hipStreamSynchronize(lst));
        bool missing = false;
        for (uint64_t i = next; i < n; ++i) missing |= res[i] == 0xFF;
        if (!missing) break;
        if (trace_qc) fprintf(stderr, "pbftv[dev %d] qc n=%llu: 2-s timeout, armed %u\n", d.id, (unsigned long long)n, cur);
        if (cur) {
          // an armed server that left without its exit being seen (no fault:
          // the streams synchronised cleanly) is a lost doorbell, not a device
          // error: serve the request with a launch instead
          cur = 0;
          std::memset(const_cast<uint8_t*>(res), 0xFF, n);
          int rc = launch_plain();
          if (rc != PBFTV_OK) return rc;
          next = 0;
          t0 = std::chrono::steady_clock::now();
          continue;
        }
        return fail(PBFTV_EDEVICE, "wave verify kernel did not report every signature");
      }
    }
    if (cur) {
      // the armed row schedule leaves an exceptional signature (a doubling or
      // cancellation in its tree, a window with two zero digits, r + n < p) to
      // the launched kernel's exact path: result byte 2 (rare; adversarial
      // inputs only)
      bool rerun = false;
      for (uint64_t i = 0; i < n; ++i) rerun |= res[i] == 2;
      if (rerun) {
        ++d.qc_reruns;
        std::memset(const_cast<uint8_t*>(res), 0xFF, n);
        int rc = launch_plain();
        if (rc != PBFTV_OK) return rc;
        HIP_TRY(hipStreamSynchronize(lst));
        for (uint64_t i = 0; i < n; ++i)
          if (res[i] == 0xFF) return fail(PBFTV_EDEVICE, "wave verify kernel did not report every signature");
      }
    }
    if (d.keeper_idle || (d.arm_seq == 0 && d.keeper.joinable())) {
      // past its keep window, or nothing armed after a larger call: the
      // keeper arms one again as soon as this call releases the device
      d.keeper_idle = false;
      d.keeper_cv.notify_one();
    }
    if (cur && d.arm_seq == 0) {  // the served number was 2^32 - 1: the kernel now waits for 0
      __atomic_store_n(&m->stop, 0u, __ATOMIC_RELEASE);
      HIP_TRY(set_dev());
      HIP_TRY(qc_disarm(d));
    }
    std::memset(out_bitmap, 0, (n + 7) / 8);
    for (uint64_t i = 0; i < n; ++i) {
      const uint8_t b = res[i];
      out_bitmap[i >> 3] |= (uint8_t)((b & 1u) << (i & 7));
      d.qc_exact_sigs += (b & pbftv::kRowsExact) ? 1u : 0u;  // a launched row kernel's exact path
    }
    d.qc_armed += cur != 0;
    const auto h_out = std::chrono::steady_clock::now();
    auto ns = [](std::chrono::steady_clock::duration x) {
      return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(x).count();
    };
    d.qc_ns_entry = ns(h_in - h_entry);
    d.qc_ns_slots = ns(h_slots - h_entry);
    d.qc_ns_handover = ns(h_bell - h_entry);
    d.qc_ns_total = ns(h_out - h_entry);
    d.qc_armed_served = cur != 0;
    return PBFTV_OK;
  }
  return run_sharded(ctx, n, [&](Device& d, Shard s) -> int {
    std::lock_guard<std::mutex> lk(d.mu);
    HIP_TRY(hipSetDevice(d.id));
    return verify_host_pipelined(d, hashes + 32 * s.lo, sig_rs + 64 * s.lo,
                                 key_idx + s.lo, s.hi - s.lo, out_bitmap + s.lo / 8);
  });
}

int pbftv_qc_stamps(pbftv_ctx* ctx, int dev, uint64_t out[8]) {
  Device* d = dev_of(ctx, dev);
  if (!d || !out) return fail(PBFTV_EINVAL, "bad context, device index or out pointer");
  std::lock_guard<std::mutex> lk(d->mu);
  std::memset(out, 0, 8 * sizeof(uint64_t));
  out[0] = d->qc_ns_handover;
  out[1] = d->qc_ns_total;
  out[2] = (d->qc_armed_served ? 1 : 0) | (std::min<uint64_t>(d->qc_ns_slots, 0x7FFFFFFFull) << 1) |
           (std::min<uint64_t>(d->qc_ns_entry, 0xFFFFFFFFull) << 32);
  if (d->qc_armed_served && d->stage.p) {
    const volatile uint64_t* st = reinterpret_cast<const volatile uint64_t*>(
        d->stage.as<uint8_t>() + QcMail::stamps_off(qc_mail(*d)->cap));
    for (int i = 0; i < 4; ++i) out[3 + i] = st[i];
  }
  int khz = 100000;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, d->id);
  out[7] = (uint64_t)khz;
  return PBFTV_OK;
}

int pbftv_qc_counters(pbftv_ctx* ctx, int dev, uint64_t out[8]) {
  Device* d = dev_of(ctx, dev);
  if (!d || !out) return fail(PBFTV_EINVAL, "bad context, device index or out pointer");
  std::lock_guard<std::mutex> lk(d->mu);
  out[0] = d->qc_calls;
  out[1] = d->qc_armed;
  out[2] = d->qc_reruns;
  out[3] = d->qc_exact_sigs;
  out[4] = d->qc_launches;
  out[5] = d->qc_armings;
  out[6] = d->rotations;
  out[7] = d->arm_seq ? (uint64_t)d->arm_waves | ((uint64_t)(d->arm_wide ? 1 : 0) << 32) : 0;
  return PBFTV_OK;
}

int pbftv_qc_stamps_all(pbftv_ctx* ctx, int dev, uint64_t* out, uint32_t waves) {
  Device* d = dev_of(ctx, dev);
  if (!d || (waves && !out)) return fail(PBFTV_EINVAL, "bad context, device index or out pointer");
  std::lock_guard<std::mutex> lk(d->mu);
  std::memset(out, 0, 4 * sizeof(uint64_t) * waves);
  if (!d->qc_armed_served || !d->stage.p) return 0;
  const volatile uint64_t* st = reinterpret_cast<const volatile uint64_t*>(
      d->stage.as<uint8_t>() + QcMail::stamps_off(qc_mail(*d)->cap));
  const uint32_t w = std::min(waves, kQcCap);
  for (uint32_t i = 0; i < 4 * w; ++i) out[i] = st[i];
  return (int)w;
}

int pbftv_qc_verify(pbftv_ctx* ctx, const uint8_t* hashes, const uint8_t* sig_rs, const uint32_t* key_idx, uint64_t n,
                    uint32_t quorum, uint8_t* out_bitmap, uint64_t* out_accepted, int* out_quorum) {
  std::vector<uint8_t> local;
  uint8_t* bm = out_bitmap;
  if (!bm) {
    local.assign((n + 7) / 8 + 1, 0);
    bm = local.data();
  }
  int rc = pbftv_ecdsa_p256_verify_batch(ctx, hashes, sig_rs, key_idx, n, bm);
  if (rc != PBFTV_OK) return rc;
  uint64_t cnt = 0;
  for (uint64_t i = 0; i < n / 8; ++i) cnt += (uint64_t)__builtin_popcount(bm[i]);
  if (n % 8) cnt += (uint64_t)__builtin_popcount(bm[n / 8] & ((1u << (n % 8)) - 1u));
  if (out_accepted) *out_accepted = cnt;
  if (out_quorum) *out_quorum = cnt >= quorum ? 1 : 0;
  return PBFTV_OK;
}

// ---------------------------------------------------------------- sha256
int pbftv_sha256_order_dev(pbftv_ctx* ctx, int dev, const uint32_t* d_lengths, uint64_t n, uint32_t* d_order,
                           void* stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return fail(PBFTV_EINVAL, "bad context or device index");
  Device& d = *ctx->devs[dev];
  std::lock_guard<std::mutex> lk(d.mu);
  HIP_TRY(hipSetDevice(d.id));
  HIP_TRY(d.order_scratch.ensure(pbftv::sha256_order_scratch_bytes(n)));
  hipStream_t st = pick_stream(d, stream);
  HIP_TRY(scratch_acquire(d, st));
  HIP_TRY(pbftv::launch_sha256_order(d_lengths, n, d_order, d.order_scratch.p, st));
  HIP_TRY(scratch_release(d, st));
  return PBFTV_OK;
}

int pbftv_sha256_batch_dev(pbftv_ctx* ctx, int dev, const uint8_t* d_data, const uint64_t* d_offsets,
                           const uint32_t* d_lengths, const uint32_t* d_order, uint64_t n, uint8_t* d_digests,
                           const uint8_t* d_expected, uint8_t* d_bitmap, void* stream) {
  if (!ctx || dev < 0 || dev >= (int)ctx->devs.size()) return fail(PBFTV_EINVAL, "bad context or device index");
  if (n && (!d_data || !d_offsets || !d_lengths || !d_digests)) return fail(PBFTV_EINVAL, "null buffer");
  if (d_expected && !d_bitmap) return fail(PBFTV_EINVAL, "expected given without bitmap");
  Device& d = *ctx->devs[dev];
  std::lock_guard<std::mutex> lk(d.mu);
  HIP_TRY(hipSetDevice(d.id));
  hipStream_t st = pick_stream(d, stream);
  HIP_TRY(timed(d, PBFTV_K_SHA256, st, [&] {
    return pbftv::launch_sha256(d_data, d_offsets, d_lengths, d_order, n, d_digests, d_expected, d_bitmap, st);
  }));
  return PBFTV_OK;
}

// Small host-buffer digest calls (utils.Hash of one request, a handful of
// messages): no DMA at all.  The messages, offsets and lengths are packed into
// pinned device-coherent host memory that k_sha256 reads over the bus, the
// digests (and match bits) come back the same way, and one launch on the
// latency stream plus its synchronisation is the whole device part -- instead
// of three copies up, the block-count sort, the kernel and a copy down
// (pbftv_hash_hex 99 B: profiles/r06_single_calls.json).
constexpr uint64_t kShaZeroCopyMsgs = 64, kShaZeroCopyBytes = 64 << 10;

static int sha_host_small(Device& d, const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths,
                          uint64_t n, uint64_t lo_b, uint64_t span, uint8_t* out_digests) {
  // layout: offsets (8n) | lengths (4n) | digests (32n) | data (span + 256: k_sha256 reads whole aligned lines)
  const uint64_t o_len = 8 * n, o_dig = o_len + 4 * n;
  const uint64_t o_data = (o_dig + 32 * n + 127) & ~127ull;
  std::lock_guard<std::mutex> lk(d.mu);
  HIP_TRY(hipSetDevice(d.id));
  HIP_TRY(d.sstage.ensure(o_data + span + 256));
  uint8_t* b = d.sstage.as<uint8_t>();
  uint64_t* off = reinterpret_cast<uint64_t*>(b);
  for (uint64_t i = 0; i < n; ++i) off[i] = offsets[i] - lo_b;
  std::memcpy(b + o_len, lengths, 4 * n);
  if (span) std::memcpy(b + o_data, data + lo_b, span);
  hipStream_t lst = nullptr;
  HIP_TRY(latency_stream(d, &lst));
  HIP_TRY(timed(d, PBFTV_K_SHA256, lst, [&] {
    return pbftv::launch_sha256(b + o_data, off, reinterpret_cast<const uint32_t*>(b + o_len), nullptr, n, b + o_dig,
                                nullptr, nullptr, lst);
  }));
  HIP_TRY(hipStreamSynchronize(lst));
  std::memcpy(out_digests, b + o_dig, 32 * n);
  return PBFTV_OK;
}

static int sha_host(pbftv_ctx* ctx, const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths,
                    const uint8_t* expected, uint64_t n, uint8_t* out_digests, uint8_t* out_bitmap) {
  if (!ctx) return fail(PBFTV_EINVAL, "ctx is null");
  if (n && (!offsets || !lengths)) return fail(PBFTV_EINVAL, "null buffer");
  if (n && n <= kShaZeroCopyMsgs && !expected) {  // (match bits: device atomics, so the DMA path)
    uint64_t lo_b = UINT64_MAX, hi_b = 0;
    for (uint64_t i = 0; i < n; ++i) {
      lo_b = std::min(lo_b, offsets[i]);
      hi_b = std::max(hi_b, offsets[i] + lengths[i]);
    }
    if (lo_b > hi_b) lo_b = hi_b;
    if (hi_b > lo_b && !data) return fail(PBFTV_EINVAL, "data is null");
    if (hi_b - lo_b <= kShaZeroCopyBytes)
      return sha_host_small(*ctx->dev0, data, offsets, lengths, n, lo_b, hi_b - lo_b, out_digests);
  }
  return run_sharded(ctx, n, [&](Device& d, Shard s) -> int {
    const uint64_t m = s.hi - s.lo;
    // byte span of this shard, re-based offsets
    uint64_t lo_b = UINT64_MAX, hi_b = 0;
    for (uint64_t i = s.lo; i < s.hi; ++i) {
      lo_b = std::min(lo_b, offsets[i]);
      hi_b = std::max(hi_b, offsets[i] + lengths[i]);
    }
    if (hi_b > lo_b && !data) return fail(PBFTV_EINVAL, "data is null");
    if (lo_b > hi_b) lo_b = hi_b;
    std::vector<uint64_t> off(m);
    for (uint64_t i = 0; i < m; ++i) off[i] = offsets[s.lo + i] - lo_b;
    const uint64_t span = hi_b - lo_b;
    std::lock_guard<std::mutex> lk(d.mu);
    HIP_TRY(hipSetDevice(d.id));
    HIP_TRY(d.data.ensure(span + 64));
    HIP_TRY(d.offsets.ensure(m * 8));
    HIP_TRY(d.lengths.ensure(m * 4));
    HIP_TRY(d.order.ensure(m * 4));
    HIP_TRY(d.digests.ensure(m * 32));
    HIP_TRY(d.order_scratch.ensure(pbftv::sha256_order_scratch_bytes(m)));
    if (span) HIP_TRY(hipMemcpyAsync(d.data.p, data + lo_b, span, hipMemcpyHostToDevice, d.stream));
    HIP_TRY(hipMemcpyAsync(d.offsets.p, off.data(), m * 8, hipMemcpyHostToDevice, d.stream));
    HIP_TRY(hipMemcpyAsync(d.lengths.p, lengths + s.lo, m * 4, hipMemcpyHostToDevice, d.stream));
    HIP_TRY(scratch_acquire(d, d.stream));
    HIP_TRY(pbftv::launch_sha256_order(d.lengths.as<uint32_t>(), m, d.order.as<uint32_t>(), d.order_scratch.p,
                                       d.stream));
    HIP_TRY(scratch_release(d, d.stream));
    uint8_t* dexp = nullptr;
    if (expected) {
      HIP_TRY(d.expected.ensure(m * 32));
      HIP_TRY(d.shabits.ensure((m + 31) / 32 * 4));
      HIP_TRY(hipMemcpyAsync(d.expected.p, expected + 32 * s.lo, m * 32, hipMemcpyHostToDevice, d.stream));
      dexp = d.expected.as<uint8_t>();
    }
    HIP_TRY(timed(d, PBFTV_K_SHA256, d.stream, [&] {
      return pbftv::launch_sha256(d.data.as<uint8_t>(), d.offsets.as<uint64_t>(), d.lengths.as<uint32_t>(),
                                  d.order.as<uint32_t>(), m, d.digests.as<uint8_t>(), dexp, d.shabits.as<uint8_t>(),
                                  d.stream);
    }));
    if (out_digests)
      HIP_TRY(hipMemcpyAsync(out_digests + 32 * s.lo, d.digests.p, m * 32, hipMemcpyDeviceToHost, d.stream));
    if (expected)
      HIP_TRY(hipMemcpyAsync(out_bitmap + s.lo / 8, d.shabits.p, (m + 7) / 8, hipMemcpyDeviceToHost, d.stream));
    HIP_TRY(hipStreamSynchronize(d.stream));
    return PBFTV_OK;
  });
}

int pbftv_sha256_batch(pbftv_ctx* ctx, const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths,
                       uint64_t n, uint8_t* out_digests) {
  if (n && !out_digests) return fail(PBFTV_EINVAL, "out_digests is null");
  return sha_host(ctx, data, offsets, lengths, nullptr, n, out_digests, nullptr);
}

int pbftv_digest_check_batch(pbftv_ctx* ctx, const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths,
                             const uint8_t* expected, uint64_t n, uint8_t* out_bitmap) {
  if (n && (!expected || !out_bitmap)) return fail(PBFTV_EINVAL, "null buffer");
  return sha_host(ctx, data, offsets, lengths, expected, n, nullptr, out_bitmap);
}

int pbftv_hash_hex(pbftv_ctx* ctx, const uint8_t* content, uint64_t len, char out_hex[65]) {
  if (!out_hex || (len && !content)) return fail(PBFTV_EINVAL, "null buffer");
  if (len > 0xFFFFFFFFull) return fail(PBFTV_EINVAL, "message longer than 4 GiB");
  uint64_t off = 0;
  uint32_t l = (uint32_t)len;
  uint8_t dg[32];
  int rc = pbftv_sha256_batch(ctx, content, &off, &l, 1, dg);
  if (rc != PBFTV_OK) return rc;
  static const char hx[] = "0123456789abcdef";  // encoding/hex: lowercase
  for (int i = 0; i < 32; ++i) {
    out_hex[2 * i] = hx[dg[i] >> 4];
    out_hex[2 * i + 1] = hx[dg[i] & 15];
  }
  out_hex[64] = 0;
  return PBFTV_OK;
}

// ---- message batches: Go-JSON built on the device, SHA-256, signatures ----
// Every entry point below is one device round trip per shard: the columns go
// up in one H2D copy (Packer), the encoder kernel writes the Go-JSON preimages,
// k_sha256 hashes them, the signature stage runs on the digests in HBM, and
// the results come back in one D2H copy.  The digest_*_batch functions are the
// flushes with no signatures.
int pbftv_flush_requests(pbftv_ctx* ctx, uint64_t n, const int64_t* timestamps, const uint8_t* client_ids,
                         const uint64_t* client_id_off, const uint32_t* client_id_len, const uint8_t* operations,
                         const uint64_t* operation_off, const uint32_t* operation_len, const int64_t* sequence_ids,
                         const uint8_t* sig_rs, const uint32_t* key_idx, const int64_t* assigned_seqs,
                         uint8_t* out_digests, uint8_t* out_sig_bitmap, uint8_t* out_consensus_digests) {
  if (!ctx) return fail(PBFTV_EINVAL, "ctx is null");
  if (n && (!timestamps || !client_id_off || !client_id_len || !operation_off || !operation_len || !sequence_ids))
    return fail(PBFTV_EINVAL, "null buffer");
  const bool sig = out_sig_bitmap != nullptr, two = out_consensus_digests != nullptr;
  if (n && sig && (!sig_rs || !key_idx)) return fail(PBFTV_EINVAL, "signatures requested without sig_rs/key_idx");
  if (n && two && !assigned_seqs) return fail(PBFTV_EINVAL, "consensus digests requested without assigned_seqs");
  if (sig && !keys_ready(ctx)) return fail(PBFTV_ENOKEYS, "pbftv_register_keys has not been called");
  return run_sharded(ctx, n, [&](Device& d, Shard s) -> int {
    const uint64_t m = s.hi - s.lo;
    Packer p;
    uint64_t pre = 0;
    auto sl = slots(s.lo, s.hi, [&](uint64_t i) {
      return pbftv::gojson::request_bound(client_id_len[i], operation_len[i]);
    }, &pre);
    const size_t o_slot = p.add_owned(two ? twice(std::move(sl), &pre) : std::move(sl));
    const size_t o_ts = p.add(timestamps + s.lo, 8 * m), o_seq = p.add(sequence_ids + s.lo, 8 * m);
    const size_t o_aseq = two ? p.add(assigned_seqs + s.lo, 8 * m) : 0;
    const auto cid = p.add_str(client_ids, client_id_off, client_id_len, s.lo, s.hi);
    const auto op = p.add_str(operations, operation_off, operation_len, s.lo, s.hi);
    const size_t o_sig = sig ? p.add(sig_rs + 64 * s.lo, 64 * m) : 0, o_key = sig ? p.add(key_idx + s.lo, 4 * m) : 0;
    std::lock_guard<std::mutex> lk(d.mu);
    HIP_TRY(hipSetDevice(d.id));
    int rc = upload(d, p);
    if (rc != PBFTV_OK) return rc;
    const pbftv::RequestCols c{at<int64_t>(d, o_ts), str_col(d, cid), str_col(d, op), at<int64_t>(d, o_seq)};
    const uint64_t* slot = at<uint64_t>(d, o_slot);
    rc = encode_and_hash(d, two ? 2 * m : m, slot, pre, [&] {
      hipError_t e = pbftv::launch_gojson_request(c, m, slot, d.data.as<uint8_t>(), d.lengths.as<uint32_t>(), d.stream);
      if (e != hipSuccess || !two) return e;
      pbftv::RequestCols c2 = c;  // StartConsensus digest: SequenceID assigned (pbft_impl.go:67-73)
      c2.seq = at<int64_t>(d, o_aseq);
      return pbftv::launch_gojson_request(c2, m, slot + m, d.data.as<uint8_t>(), d.lengths.as<uint32_t>() + m,
                                          d.stream);
    });
    if (rc != PBFTV_OK) return rc;
    if (sig) {
      HIP_TRY(d.bitmap.ensure((m + 7) / 8 + 8));
      rc = verify_on_device(d, d.digests.as<uint8_t>(), at<uint8_t>(d, o_sig), at<uint32_t>(d, o_key), m,
                            d.bitmap.as<uint8_t>(), d.stream);
      if (rc != PBFTV_OK) return rc;
    }
    return results_out(d, s.lo, m, {{kDigests, d.digests.p, out_digests},
                                    {kDigests, d.digests.as<uint8_t>() + 32 * m, out_consensus_digests},
                                    {kBitmap, d.bitmap.p, sig ? out_sig_bitmap : nullptr}});
  });
}

int pbftv_digest_request_batch(pbftv_ctx* ctx, uint64_t n, const int64_t* timestamps, const uint8_t* client_ids,
                               const uint64_t* client_id_off, const uint32_t* client_id_len, const uint8_t* operations,
                               const uint64_t* operation_off, const uint32_t* operation_len,
                               const int64_t* sequence_ids, uint8_t* out_digests) {
  if (n && !out_digests) return fail(PBFTV_EINVAL, "null buffer");
  return pbftv_flush_requests(ctx, n, timestamps, client_ids, client_id_off, client_id_len, operations, operation_off,
                              operation_len, sequence_ids, nullptr, nullptr, nullptr, out_digests, nullptr, nullptr);
}

int pbftv_digest_vote_batch(pbftv_ctx* ctx, uint64_t n, const int64_t* view_ids, const int64_t* sequence_ids,
                            const uint8_t* digests, const uint64_t* digest_off, const uint32_t* digest_len,
                            const uint8_t* node_ids, const uint64_t* node_id_off, const uint32_t* node_id_len,
                            const int64_t* msg_types, uint8_t* out_digests) {
  if (n && !out_digests) return fail(PBFTV_EINVAL, "null buffer");
  return pbftv_flush_votes(ctx, n, view_ids, sequence_ids, digests, digest_off, digest_len, node_ids, node_id_off,
                           node_id_len, msg_types, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr,
                           out_digests, nullptr, nullptr);
}

int pbftv_flush_replies(pbftv_ctx* ctx, uint64_t n, const int64_t* view_ids, const int64_t* timestamps,
                        const uint8_t* client_ids, const uint64_t* client_id_off, const uint32_t* client_id_len,
                        const uint8_t* node_ids, const uint64_t* node_id_off, const uint32_t* node_id_len,
                        const uint8_t* results, const uint64_t* result_off, const uint32_t* result_len,
                        const uint8_t* sig_rs, const uint32_t* key_idx, uint8_t* out_digests,
                        uint8_t* out_sig_bitmap) {
  if (!ctx) return fail(PBFTV_EINVAL, "ctx is null");
  if (n && (!view_ids || !timestamps || !client_id_off || !client_id_len || !node_id_off || !node_id_len ||
            !result_off || !result_len))
    return fail(PBFTV_EINVAL, "null buffer");
  const bool sig = out_sig_bitmap != nullptr;
  if (n && sig && (!sig_rs || !key_idx)) return fail(PBFTV_EINVAL, "signatures requested without sig_rs/key_idx");
  if (sig && !keys_ready(ctx)) return fail(PBFTV_ENOKEYS, "pbftv_register_keys has not been called");
  return run_sharded(ctx, n, [&](Device& d, Shard s) -> int {
    const uint64_t m = s.hi - s.lo;
    Packer p;
    uint64_t pre = 0;
    const size_t o_slot = p.add_owned(slots(s.lo, s.hi, [&](uint64_t i) {
      return pbftv::gojson::reply_bound(client_id_len[i], node_id_len[i], result_len[i]);
    }, &pre));
    const size_t o_view = p.add(view_ids + s.lo, 8 * m), o_ts = p.add(timestamps + s.lo, 8 * m);
    const auto cid = p.add_str(client_ids, client_id_off, client_id_len, s.lo, s.hi);
    const auto nid = p.add_str(node_ids, node_id_off, node_id_len, s.lo, s.hi);
    const auto res = p.add_str(results, result_off, result_len, s.lo, s.hi);
    const size_t o_sig = sig ? p.add(sig_rs + 64 * s.lo, 64 * m) : 0, o_key = sig ? p.add(key_idx + s.lo, 4 * m) : 0;
    std::lock_guard<std::mutex> lk(d.mu);
    HIP_TRY(hipSetDevice(d.id));
    int rc = upload(d, p);
    if (rc != PBFTV_OK) return rc;
    const pbftv::ReplyCols c{at<int64_t>(d, o_view), at<int64_t>(d, o_ts), str_col(d, cid), str_col(d, nid),
                             str_col(d, res)};
    const uint64_t* slot = at<uint64_t>(d, o_slot);
    rc = encode_and_hash(d, m, slot, pre, [&] {
      return pbftv::launch_gojson_reply(c, m, slot, d.data.as<uint8_t>(), d.lengths.as<uint32_t>(), d.stream);
    });
    if (rc != PBFTV_OK) return rc;
    if (sig) {
      HIP_TRY(d.bitmap.ensure((m + 7) / 8 + 8));
      rc = verify_on_device(d, d.digests.as<uint8_t>(), at<uint8_t>(d, o_sig), at<uint32_t>(d, o_key), m,
                            d.bitmap.as<uint8_t>(), d.stream);
      if (rc != PBFTV_OK) return rc;
    }
    return results_out(d, s.lo, m, {{kDigests, d.digests.p, out_digests},
                                    {kBitmap, d.bitmap.p, sig ? out_sig_bitmap : nullptr}});
  });
}

int pbftv_digest_reply_batch(pbftv_ctx* ctx, uint64_t n, const int64_t* view_ids, const int64_t* timestamps,
                             const uint8_t* client_ids, const uint64_t* client_id_off, const uint32_t* client_id_len,
                             const uint8_t* node_ids, const uint64_t* node_id_off, const uint32_t* node_id_len,
                             const uint8_t* results, const uint64_t* result_off, const uint32_t* result_len,
                             uint8_t* out_digests) {
  if (n && !out_digests) return fail(PBFTV_EINVAL, "null buffer");
  return pbftv_flush_replies(ctx, n, view_ids, timestamps, client_ids, client_id_off, client_id_len, node_ids,
                             node_id_off, node_id_len, results, result_off, result_len, nullptr, nullptr, out_digests,
                             nullptr);
}

int pbftv_flush_preprepares(pbftv_ctx* ctx, uint64_t n, const int64_t* view_ids, const int64_t* sequence_ids,
                            const uint8_t* digests, const uint64_t* digest_off, const uint32_t* digest_len,
                            const uint8_t* has_request, const int64_t* req_timestamps, const uint8_t* req_client_ids,
                            const uint64_t* req_client_id_off, const uint32_t* req_client_id_len,
                            const uint8_t* req_operations, const uint64_t* req_operation_off,
                            const uint32_t* req_operation_len, const int64_t* req_sequence_ids, const uint8_t* sig_rs,
                            const uint32_t* key_idx, uint32_t n_states, const int64_t* state_view_ids,
                            const int64_t* state_last_seqs, const uint32_t* state_idx, uint8_t* out_digests,
                            uint8_t* out_req_digests, uint8_t* out_sig_bitmap, uint8_t* out_msg_bitmap) {
  if (!ctx) return fail(PBFTV_EINVAL, "ctx is null");
  if (n && (!view_ids || !sequence_ids || !digest_off || !digest_len || !has_request || !req_timestamps ||
            !req_client_id_off || !req_client_id_len || !req_operation_off || !req_operation_len ||
            !req_sequence_ids))
    return fail(PBFTV_EINVAL, "null buffer");
  const bool sig = out_sig_bitmap != nullptr, msg = out_msg_bitmap != nullptr;
  if (n && sig && (!sig_rs || !key_idx)) return fail(PBFTV_EINVAL, "signatures requested without sig_rs/key_idx");
  if (n && msg && (!state_idx || (n_states && (!state_view_ids || !state_last_seqs))))
    return fail(PBFTV_EINVAL, "verifyMsg requested without states");
  if (sig && !keys_ready(ctx)) return fail(PBFTV_ENOKEYS, "pbftv_register_keys has not been called");
  // the embedded requests' digests are needed for verifyMsg or when asked for
  const bool pair = msg || out_req_digests != nullptr;
  return run_sharded(ctx, n, [&](Device& d, Shard s) -> int {
    const uint64_t m = s.hi - s.lo;
    Packer p;
    uint64_t pre = 0;
    auto rb = [&](uint64_t i) {
      return has_request[i] ? pbftv::gojson::request_bound(req_client_id_len[i], req_operation_len[i]) : 4;
    };
    auto sl = slots(s.lo, s.hi, [&](uint64_t i) {
      return pbftv::gojson::preprepare_bound(digest_len[i], has_request[i] ? req_client_id_len[i] : 0,
                                             has_request[i] ? req_operation_len[i] : 0);
    }, &pre);
    if (pair) {  // request preimages in slots [m, 2m)
      uint64_t pre2 = 0;
      auto s2 = slots(s.lo, s.hi, rb, &pre2);
      sl.resize(2 * m);
      for (uint64_t i = 0; i < m; ++i) sl[m + i] = pre + s2[i];
      pre += pre2;
    }
    const size_t o_slot = p.add_owned(std::move(sl));
    const size_t o_view = p.add(view_ids + s.lo, 8 * m), o_seq = p.add(sequence_ids + s.lo, 8 * m);
    const size_t o_has = p.add(has_request + s.lo, m);
    const size_t o_rts = p.add(req_timestamps + s.lo, 8 * m), o_rseq = p.add(req_sequence_ids + s.lo, 8 * m);
    const auto dg = p.add_str(digests, digest_off, digest_len, s.lo, s.hi);
    const auto cid = p.add_str(req_client_ids, req_client_id_off, req_client_id_len, s.lo, s.hi);
    const auto op = p.add_str(req_operations, req_operation_off, req_operation_len, s.lo, s.hi);
    const size_t o_sig = sig ? p.add(sig_rs + 64 * s.lo, 64 * m) : 0, o_key = sig ? p.add(key_idx + s.lo, 4 * m) : 0;
    size_t o_sv = 0, o_sl = 0, o_si = 0;
    if (msg) {
      o_sv = p.add(state_view_ids, 8ull * n_states);
      o_sl = p.add(state_last_seqs, 8ull * n_states);
      o_si = p.add(state_idx + s.lo, 4 * m);
    }
    std::lock_guard<std::mutex> lk(d.mu);
    HIP_TRY(hipSetDevice(d.id));
    int rc = upload(d, p);
    if (rc != PBFTV_OK) return rc;
    const pbftv::PrePrepareCols c{
        at<int64_t>(d, o_view), at<int64_t>(d, o_seq), str_col(d, dg), at<uint8_t>(d, o_has),
        {at<int64_t>(d, o_rts), str_col(d, cid), str_col(d, op), at<int64_t>(d, o_rseq)}};
    const uint64_t* slot = at<uint64_t>(d, o_slot);
    rc = encode_and_hash(d, pair ? 2 * m : m, slot, pre, [&] {
      return pair ? pbftv::launch_gojson_preprepare_pair(c, m, slot, d.data.as<uint8_t>(), d.lengths.as<uint32_t>(),
                                                         d.stream)
                  : pbftv::launch_gojson_preprepare(c, m, slot, d.data.as<uint8_t>(), d.lengths.as<uint32_t>(),
                                                    d.stream);
    });
    if (rc != PBFTV_OK) return rc;
    if (sig) {
      HIP_TRY(d.bitmap.ensure((m + 7) / 8 + 8));
      rc = verify_on_device(d, d.digests.as<uint8_t>(), at<uint8_t>(d, o_sig), at<uint32_t>(d, o_key), m,
                            d.bitmap.as<uint8_t>(), d.stream);
      if (rc != PBFTV_OK) return rc;
    }
    uint8_t* msgok = nullptr;
    if (msg) {
      HIP_TRY(d.msgok.ensure(m + 8));
      msgok = d.msgok.as<uint8_t>();
      const pbftv::StateCols sc{at<int64_t>(d, o_sv), at<int64_t>(d, o_sl), nullptr, at<uint32_t>(d, o_si), n_states};
      HIP_TRY(pbftv::launch_preprepare_verify(c.view, c.seq, c.digest, d.digests.as<uint8_t>() + 32 * m, sc, m, msgok,
                                             d.stream));
    }
    return results_out(d, s.lo, m, {{kDigests, d.digests.p, out_digests},
                                    {kDigests, d.digests.as<uint8_t>() + 32 * m, pair ? out_req_digests : nullptr},
                                    {kBitmap, d.bitmap.p, sig ? out_sig_bitmap : nullptr},
                                    {kByteFlags, msgok, out_msg_bitmap}});
  });
}

int pbftv_digest_preprepare_batch(pbftv_ctx* ctx, uint64_t n, const int64_t* view_ids, const int64_t* sequence_ids,
                                  const uint8_t* digests, const uint64_t* digest_off, const uint32_t* digest_len,
                                  const uint8_t* has_request, const int64_t* req_timestamps,
                                  const uint8_t* req_client_ids, const uint64_t* req_client_id_off,
                                  const uint32_t* req_client_id_len, const uint8_t* req_operations,
                                  const uint64_t* req_operation_off, const uint32_t* req_operation_len,
                                  const int64_t* req_sequence_ids, uint8_t* out_digests) {
  if (n && !out_digests) return fail(PBFTV_EINVAL, "null buffer");
  return pbftv_flush_preprepares(ctx, n, view_ids, sequence_ids, digests, digest_off, digest_len, has_request,
                                 req_timestamps, req_client_ids, req_client_id_off, req_client_id_len, req_operations,
                                 req_operation_off, req_operation_len, req_sequence_ids, nullptr, nullptr, 0, nullptr,
                                 nullptr, nullptr, out_digests, nullptr, nullptr, nullptr);
}

// Pool flush of a vote snapshot: Go-JSON + SHA-256 + verifyMsg + ECDSA in one
// device round trip per shard (see pbftv.h).  Also the body of
// pbftv_digest_vote_batch (no signatures, no states).
int pbftv_flush_votes(pbftv_ctx* ctx, uint64_t n, const int64_t* view_ids, const int64_t* sequence_ids,
                      const uint8_t* digests, const uint64_t* digest_off, const uint32_t* digest_len,
                      const uint8_t* node_ids, const uint64_t* node_id_off, const uint32_t* node_id_len,
                      const int64_t* msg_types, const uint8_t* sig_rs, const uint32_t* key_idx, uint32_t n_states,
                      const int64_t* state_view_ids, const int64_t* state_last_seqs,
                      const uint8_t* state_req_digests, const uint32_t* state_idx, uint8_t* out_digests,
                      uint8_t* out_sig_bitmap, uint8_t* out_msg_bitmap) {
  if (!ctx) return fail(PBFTV_EINVAL, "ctx is null");
  if (n && (!view_ids || !sequence_ids || !digest_off || !digest_len || !node_id_off || !node_id_len || !msg_types))
    return fail(PBFTV_EINVAL, "null buffer");
  const bool sig = out_sig_bitmap != nullptr, msg = out_msg_bitmap != nullptr;
  if (n && sig && (!sig_rs || !key_idx)) return fail(PBFTV_EINVAL, "signatures requested without sig_rs/key_idx");
  if (n && msg && (!state_idx || (n_states && (!state_view_ids || !state_last_seqs || !state_req_digests))))
    return fail(PBFTV_EINVAL, "verifyMsg requested without states");
  if (sig && !keys_ready(ctx)) return fail(PBFTV_ENOKEYS, "pbftv_register_keys has not been called");
  return run_sharded(ctx, n, [&](Device& d, Shard s) -> int {
    const uint64_t m = s.hi - s.lo;
    Packer p;
    uint64_t pre = 0;
    const size_t o_slot = p.add_owned(slots(s.lo, s.hi, [&](uint64_t i) {
      return pbftv::gojson::vote_bound(digest_len[i], node_id_len[i]);
    }, &pre));
    const size_t o_view = p.add(view_ids + s.lo, 8 * m), o_seq = p.add(sequence_ids + s.lo, 8 * m),
                 o_type = p.add(msg_types + s.lo, 8 * m);
    const auto dg = p.add_str(digests, digest_off, digest_len, s.lo, s.hi);
    const auto nid = p.add_str(node_ids, node_id_off, node_id_len, s.lo, s.hi);
    size_t o_sig = 0, o_key = 0, o_sv = 0, o_sl = 0, o_sd = 0, o_si = 0;
    if (sig) {
      o_sig = p.add(sig_rs + 64 * s.lo, 64 * m);
      o_key = p.add(key_idx + s.lo, 4 * m);
    }
    if (msg) {
      o_sv = p.add(state_view_ids, 8ull * n_states);
      o_sl = p.add(state_last_seqs, 8ull * n_states);
      o_sd = p.add(state_req_digests, 32ull * n_states);
      o_si = p.add(state_idx + s.lo, 4 * m);
    }
    std::lock_guard<std::mutex> lk(d.mu);
    HIP_TRY(hipSetDevice(d.id));
    int rc = upload(d, p);
    if (rc != PBFTV_OK) return rc;
    const pbftv::VoteCols c{at<int64_t>(d, o_view), at<int64_t>(d, o_seq), str_col(d, dg), str_col(d, nid),
                            at<int64_t>(d, o_type)};
    pbftv::StateCols sc{nullptr, nullptr, nullptr, nullptr, n_states};
    uint8_t* msgok = nullptr;
    if (msg) {
      sc = {at<int64_t>(d, o_sv), at<int64_t>(d, o_sl), at<uint8_t>(d, o_sd), at<uint32_t>(d, o_si), n_states};
      HIP_TRY(d.msgok.ensure(m + 8));
      msgok = d.msgok.as<uint8_t>();
    }
    const uint64_t* slot = at<uint64_t>(d, o_slot);
    rc = encode_and_hash(d, m, slot, pre, [&] {
      return pbftv::launch_gojson_vote(c, m, slot, d.data.as<uint8_t>(), d.lengths.as<uint32_t>(), sc, msgok,
                                       d.stream);
    });
    if (rc != PBFTV_OK) return rc;
    if (sig) {
      HIP_TRY(d.bitmap.ensure((m + 7) / 8 + 8));
      rc = verify_on_device(d, d.digests.as<uint8_t>(), at<uint8_t>(d, o_sig), at<uint32_t>(d, o_key), m,
                            d.bitmap.as<uint8_t>(), d.stream);
      if (rc != PBFTV_OK) return rc;
    }
    return results_out(d, s.lo, m, {{kDigests, d.digests.p, out_digests},
                                    {kBitmap, d.bitmap.p, sig ? out_sig_bitmap : nullptr},
                                    {kByteFlags, msgok, out_msg_bitmap}});
  });
}

int pbftv_verify_msg_batch(int64_t state_view_id, int64_t state_last_seq, const uint8_t req_digest[32], uint64_t n,
                           const int64_t* view_ids, const int64_t* sequence_ids, const char* digest_got,
                           const uint64_t* digest_got_off, const uint32_t* digest_got_len, uint8_t* out_bitmap) {
  if (!req_digest || (n && (!view_ids || !sequence_ids || !digest_got_off || !digest_got_len || !out_bitmap)))
    return fail(PBFTV_EINVAL, "null buffer");
  static const char hx[] = "0123456789abcdef";
  char want[64];
  for (int i = 0; i < 32; ++i) {
    want[2 * i] = hx[req_digest[i] >> 4];
    want[2 * i + 1] = hx[req_digest[i] & 15];
  }
  std::memset(out_bitmap, 0, (n + 7) / 8);
  for (uint64_t i = 0; i < n; ++i) {
    bool ok = view_ids[i] == state_view_id;                                  // pbft_impl.go:178
    if (ok && state_last_seq != -1) ok = state_last_seq < sequence_ids[i];    // pbft_impl.go:184-188
    ok = ok && digest_got_len[i] == 64 && digest_got &&                       // pbft_impl.go:197 string compare
         std::memcmp(digest_got + digest_got_off[i], want, 64) == 0;
    if (ok) out_bitmap[i / 8] |= (uint8_t)(1u << (i % 8));
  }
  return PBFTV_OK;
}

uint64_t pbftv_gojson_request(int64_t timestamp, const char* client_id, uint64_t client_id_len, const char* operation,
                              uint64_t operation_len, int64_t sequence_id, uint8_t* out, uint64_t cap) {
  std::vector<uint8_t> b;
  pbftv::gojson::append_request(b, timestamp, reinterpret_cast<const uint8_t*>(client_id), client_id_len,
                                reinterpret_cast<const uint8_t*>(operation), operation_len, sequence_id);
  if (out) std::memcpy(out, b.data(), std::min<uint64_t>(cap, b.size()));
  return b.size();
}

uint64_t pbftv_gojson_vote(int64_t view_id, int64_t sequence_id, const char* digest, uint64_t digest_len,
                           const char* node_id, uint64_t node_id_len, int64_t msg_type, uint8_t* out, uint64_t cap) {
  std::vector<uint8_t> b;
  pbftv::gojson::append_vote(b, view_id, sequence_id, reinterpret_cast<const uint8_t*>(digest), digest_len,
                             reinterpret_cast<const uint8_t*>(node_id), node_id_len, msg_type);
  if (out) std::memcpy(out, b.data(), std::min<uint64_t>(cap, b.size()));
  return b.size();
}

uint64_t pbftv_gojson_vote_signed(int64_t view_id, int64_t sequence_id, const char* digest, uint64_t digest_len,
                                  const char* node_id, uint64_t node_id_len, int64_t msg_type, const uint8_t* sig,
                                  uint64_t sig_len, int sig_nil, uint8_t* out, uint64_t cap) {
  std::vector<uint8_t> b;
  pbftv::gojson::append_vote_signed(b, view_id, sequence_id, reinterpret_cast<const uint8_t*>(digest), digest_len,
                                    reinterpret_cast<const uint8_t*>(node_id), node_id_len, msg_type, sig, sig_len,
                                    sig_nil != 0);
  if (out) std::memcpy(out, b.data(), std::min<uint64_t>(cap, b.size()));
  return b.size();
}

static pbftv::gojson::SigField sig_field(const uint8_t* sig, uint64_t sig_len, int sig_nil) {
  return {sig, sig_len, sig_nil != 0};
}

uint64_t pbftv_gojson_request_signed(int64_t timestamp, const char* client_id, uint64_t client_id_len,
                                     const char* operation, uint64_t operation_len, int64_t sequence_id,
                                     const uint8_t* sig, uint64_t sig_len, int sig_nil, uint8_t* out, uint64_t cap) {
  std::vector<uint8_t> b;
  pbftv::gojson::append_request_signed(b, timestamp, reinterpret_cast<const uint8_t*>(client_id), client_id_len,
                                       reinterpret_cast<const uint8_t*>(operation), operation_len, sequence_id,
                                       sig_field(sig, sig_len, sig_nil));
  if (out) std::memcpy(out, b.data(), std::min<uint64_t>(cap, b.size()));
  return b.size();
}

uint64_t pbftv_gojson_reply_signed(int64_t view_id, int64_t timestamp, const char* client_id, uint64_t client_id_len,
                                   const char* node_id, uint64_t node_id_len, const char* result, uint64_t result_len,
                                   const uint8_t* sig, uint64_t sig_len, int sig_nil, uint8_t* out, uint64_t cap) {
  std::vector<uint8_t> b;
  pbftv::gojson::append_reply_signed(b, view_id, timestamp, reinterpret_cast<const uint8_t*>(client_id),
                                     client_id_len, reinterpret_cast<const uint8_t*>(node_id), node_id_len,
                                     reinterpret_cast<const uint8_t*>(result), result_len,
                                     sig_field(sig, sig_len, sig_nil));
  if (out) std::memcpy(out, b.data(), std::min<uint64_t>(cap, b.size()));
  return b.size();
}

uint64_t pbftv_gojson_preprepare_signed(int64_t view_id, int64_t sequence_id, const char* digest, uint64_t digest_len,
                                        int has_request, int64_t req_timestamp, const char* req_client_id,
                                        uint64_t req_client_id_len, const char* req_operation,
                                        uint64_t req_operation_len, int64_t req_sequence_id, const uint8_t* req_sig,
                                        uint64_t req_sig_len, int req_sig_nil, const uint8_t* sig, uint64_t sig_len,
                                        int sig_nil, uint8_t* out, uint64_t cap) {
  std::vector<uint8_t> b;
  pbftv::gojson::append_preprepare_signed(
      b, view_id, sequence_id, reinterpret_cast<const uint8_t*>(digest), digest_len, has_request != 0, req_timestamp,
      reinterpret_cast<const uint8_t*>(req_client_id), req_client_id_len,
      reinterpret_cast<const uint8_t*>(req_operation), req_operation_len, req_sequence_id,
      sig_field(req_sig, req_sig_len, req_sig_nil), sig_field(sig, sig_len, sig_nil));
  if (out) std::memcpy(out, b.data(), std::min<uint64_t>(cap, b.size()));
  return b.size();
}

uint64_t pbftv_gojson_reply(int64_t view_id, int64_t timestamp, const char* client_id, uint64_t client_id_len,
                            const char* node_id, uint64_t node_id_len, const char* result, uint64_t result_len,
                            uint8_t* out, uint64_t cap) {
  std::vector<uint8_t> b;
  pbftv::gojson::append_reply(b, view_id, timestamp, reinterpret_cast<const uint8_t*>(client_id), client_id_len,
                              reinterpret_cast<const uint8_t*>(node_id), node_id_len,
                              reinterpret_cast<const uint8_t*>(result), result_len);
  if (out) std::memcpy(out, b.data(), std::min<uint64_t>(cap, b.size()));
  return b.size();
}

uint64_t pbftv_gojson_preprepare(int64_t view_id, int64_t sequence_id, const char* digest, uint64_t digest_len,
                                 int has_request, int64_t req_timestamp, const char* req_client_id,
                                 uint64_t req_client_id_len, const char* req_operation, uint64_t req_operation_len,
                                 int64_t req_sequence_id, uint8_t* out, uint64_t cap) {
  std::vector<uint8_t> b;
  pbftv::gojson::append_preprepare(b, view_id, sequence_id, reinterpret_cast<const uint8_t*>(digest), digest_len,
                                   has_request != 0, req_timestamp, reinterpret_cast<const uint8_t*>(req_client_id),
                                   req_client_id_len, reinterpret_cast<const uint8_t*>(req_operation),
                                   req_operation_len, req_sequence_id);
  if (out) std::memcpy(out, b.data(), std::min<uint64_t>(cap, b.size()));
  return b.size();
}

}  // extern "C"
