// pbft.h -- C++ mirror of the reference's consensus / pool interface for the
// crypto hot path, driving the MI355X batch verifier.
//
// The reference is Go (1556174776/simple_pbft); Go is not available here, so
// this is the host side above the C ABI, mirroring the reference's names,
// argument meaning and error strings so the tests read like the reference's
// own call sites:
//   pbft/consensus/pbft_msg_types.go:3-38   RequestMsg, ReplyMsg, PrePrepareMsg, VoteMsg, MsgType
//   pbft/consensus/pbft_impl.go:12-243      State, CreateState, StartConsensus, PrePrepare,
//                                           Prepare, Commit, verifyMsg, prepared, committed, digest
//   utils/utils.go:13-17                    Hash
//   pool/*.go                               RequestMsgPool ... ReplyMsgPool (Add/Del/DelAll/MsgNum/GetAll)
// Build-added (the author's plan, 需要改进的地方.md:17): every message carries
// a 64-byte P-256 signature r||s over SHA-256 of its Go-JSON encoding WITHOUT
// the signature, and a KeyTable maps node / client IDs to registered keys.
// The *Batch methods are the GPU flush of a whole pool snapshot
// (pbft/network/node.go:365-439, 559-598): every message of the snapshot is
// verified in one call, then applied in order with the reference's
// semantics (a vote is stored by NodeID; quorum >= 2f; processing of the
// snapshot stops once the stage advances, like the MSGENOUGH break).
#pragma once
#include <array>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <optional>
#include <shared_mutex>
#include <string>
#include <vector>

struct pbftv_ctx;

namespace pbft {

using Sig = std::array<uint8_t, 64>;
using Digest32 = std::array<uint8_t, 32>;

// ---- pbft_msg_types.go ----
struct RequestMsg {
  int64_t Timestamp = 0;
  std::string ClientID;
  std::string Operation;
  int64_t SequenceID = 0;
  Sig Signature{};
};

struct ReplyMsg {
  int64_t ViewID = 0;
  int64_t Timestamp = 0;
  std::string ClientID;
  std::string NodeID;
  std::string Result;
  Sig Signature{};
};

struct PrePrepareMsg {
  int64_t ViewID = 0;
  int64_t SequenceID = 0;
  std::string Digest;
  std::optional<RequestMsg> Request;  // *RequestMsg (nil -> null)
  std::string NodeID;                 // build-added: the signer (primary)
  Sig Signature{};
};

enum MsgType : int64_t { PrepareMsg = 0, CommitMsg = 1 };

struct VoteMsg {
  int64_t ViewID = 0;
  int64_t SequenceID = 0;
  std::string Digest;
  std::string NodeID;
  MsgType Type = PrepareMsg;
  Sig Signature{};
};

enum class Stage { Idle, PrePrepared, Prepared, Committed };

constexpr int f = 1;  // pbft_impl.go:37

// Go-JSON signing/digest preimages (json.Marshal of the reference struct, no signature)
std::vector<uint8_t> Marshal(const RequestMsg& m);
std::vector<uint8_t> Marshal(const VoteMsg& m);
std::vector<uint8_t> Marshal(const ReplyMsg& m);
std::vector<uint8_t> Marshal(const PrePrepareMsg& m);

// ---- crypto backend ---------------------------------------------------
// The product backend is GpuCrypto (the pbftv C ABI); tests may inject a
// double to exercise the state machine without a GPU.
class Crypto {
 public:
  virtual ~Crypto() = default;
  virtual std::vector<Digest32> Sha256(const std::vector<std::vector<uint8_t>>& msgs) = 0;
  // ECDSA-P256 over 32-byte hashes, keys by registered index; bit per item
  virtual std::vector<bool> Verify(const std::vector<Digest32>& hashes, const std::vector<Sig>& sigs,
                                   const std::vector<uint32_t>& key_idx) = 0;
  virtual void RegisterKeys(const std::vector<std::array<uint8_t, 64>>& pub_xy) = 0;
  // One pool flush over votes addressed to several consensus states (state i =
  // view, last sequence, 32-B request digest): sig_ok[j] = valid signature by
  // key_idx[j] over SHA-256(Marshal(votes[j])); msg_ok[j] = verifyMsg against
  // states[state_idx[j]].  The default composes Sha256 + Verify + a host
  // verifyMsg; GpuCrypto does it in one device round trip (pbftv_flush_votes).
  struct StateRef {
    int64_t view, last_seq;
    Digest32 req_digest;
  };
  virtual void FlushVotes(const std::vector<VoteMsg>& votes, const std::vector<uint32_t>& key_idx,
                          const std::vector<StateRef>& states, const std::vector<uint32_t>& state_idx,
                          std::vector<bool>& sig_ok, std::vector<bool>& msg_ok);
};

class GpuCrypto : public Crypto {
 public:
  explicit GpuCrypto(uint32_t device_mask = 0);  // throws std::runtime_error without a gfx950 GPU
  ~GpuCrypto() override;
  std::vector<Digest32> Sha256(const std::vector<std::vector<uint8_t>>& msgs) override;
  std::vector<bool> Verify(const std::vector<Digest32>& hashes, const std::vector<Sig>& sigs,
                           const std::vector<uint32_t>& key_idx) override;
  void RegisterKeys(const std::vector<std::array<uint8_t, 64>>& pub_xy) override;
  void FlushVotes(const std::vector<VoteMsg>& votes, const std::vector<uint32_t>& key_idx,
                  const std::vector<StateRef>& states, const std::vector<uint32_t>& state_idx,
                  std::vector<bool>& sig_ok, std::vector<bool>& msg_ok) override;
  pbftv_ctx* ctx() const { return ctx_; }

 private:
  pbftv_ctx* ctx_ = nullptr;
};

// utils.Hash: lowercase hex SHA-256 (utils/utils.go:13-17)
std::string Hash(Crypto& c, const std::vector<uint8_t>& content);
// digest(object) = Hash(json.Marshal(object)) (pbft_impl.go:235-243)
std::string digest(Crypto& c, const RequestMsg& r);
std::string ToHex(const Digest32& d);

// ID -> registered key index (nodes and clients); absent IDs fail verification.
class KeyTable {
 public:
  void Add(const std::string& id, uint32_t index) { idx_[id] = index; }
  std::optional<uint32_t> Find(const std::string& id) const {
    auto it = idx_.find(id);
    if (it == idx_.end()) return std::nullopt;
    return it->second;
  }

 private:
  std::map<std::string, uint32_t> idx_;
};

// Signature check of a batch of messages: one SHA-256 batch over the preimages,
// one ECDSA batch.  out[i] = valid signature by the named signer.
std::vector<bool> VerifySignatures(Crypto& c, const KeyTable& keys, const std::vector<VoteMsg>& votes);
std::vector<bool> VerifySignatures(Crypto& c, const KeyTable& keys, const std::vector<ReplyMsg>& replies);
std::vector<bool> VerifySignatures(Crypto& c, const KeyTable& keys, const std::vector<PrePrepareMsg>& pps);
std::vector<bool> VerifySignatures(Crypto& c, const KeyTable& keys, const std::vector<RequestMsg>& reqs);

// ---- pbft_impl.go ----------------------------------------------------
struct MsgLogs {
  std::optional<RequestMsg> ReqMsg;
  std::map<std::string, VoteMsg> PrepareMsgs;  // key: NodeID
  std::map<std::string, VoteMsg> CommitMsgs;
};

// Go's (value, error) pairs: ok == err.empty()
template <class T>
struct Result {
  std::optional<T> value;
  std::string err;
};

struct BatchOutcome {
  std::vector<bool> accepted;          // per snapshot item: passed signature + verifyMsg
  std::vector<std::string> errors;     // the reference's error for each rejected item
  size_t applied = 0;                  // items stored before the stage advanced (MSGENOUGH)
};

class State {
 public:
  int64_t ViewID = 0;
  MsgLogs MsgLogs_;
  int64_t LastSequenceID = -1;
  Stage CurrentStage = Stage::Idle;

  static State CreateState(int64_t viewID, int64_t lastSequenceID);  // pbft_impl.go:41-52

  // pbft_impl.go:55-88; now_unix_nano stands in for time.Now().UnixNano()
  Result<PrePrepareMsg> StartConsensus(Crypto& c, RequestMsg& request, int64_t now_unix_nano);
  // pbft_impl.go:91-109
  Result<VoteMsg> PrePrepare(Crypto& c, const PrePrepareMsg& pp);
  // pbft_impl.go:115-139: returns a commit vote once prepared()
  Result<VoteMsg> Prepare(Crypto& c, const VoteMsg& prepareMsg);
  // pbft_impl.go:145-173: returns (reply, committed request) once committed()
  Result<std::pair<ReplyMsg, RequestMsg>> Commit(Crypto& c, const VoteMsg& commitMsg);

  // GPU flush of a pool snapshot (signatures + verifyMsg for every vote in two batches)
  Result<VoteMsg> PrepareBatch(Crypto& c, const KeyTable& keys, const std::vector<VoteMsg>& snapshot,
                               BatchOutcome* outcome = nullptr);
  Result<std::pair<ReplyMsg, RequestMsg>> CommitBatch(Crypto& c, const KeyTable& keys,
                                                      const std::vector<VoteMsg>& snapshot,
                                                      BatchOutcome* outcome = nullptr);

  bool verifyMsg(Crypto& c, int64_t viewID, int64_t sequenceID, const std::string& digestGot);  // :176-202
  bool prepared() const;   // :207-217
  bool committed() const;  // :222-232

 private:
  friend class ConsensusTable;
  std::optional<std::string> req_digest_;  // digest(ReqMsg), computed once per request
  const std::string& request_digest(Crypto& c);
  std::vector<bool> verify_votes(Crypto& c, const KeyTable& keys, const std::vector<VoteMsg>& snap,
                                 std::vector<std::string>& errs, const char* what);
};

// ---- sequence-keyed concurrent consensus -------------
// The reference runs ONE State per node (node.go:277-296) and keys its vote
// pools by NodeID, so a flush sees at most n-1 votes.  The author's plan
// (需要改进的地方.md:14-24) keeps a State per sequence in flight and pools keyed
// by (sequenceID, NodeID); then one flush covers 2f*k votes of k sequences:
// ONE Crypto::FlushVotes batch (GPU: Go-JSON + SHA-256 + verifyMsg + ECDSA),
// after which each vote is applied to its own sequence's State in snapshot
// order with the reference's rules (store by NodeID, quorum 2f, the state
// stops taking votes once it advances -- MSGENOUGH, node.go:564-566).
class ConsensusTable {
 public:
  explicit ConsensusTable(int64_t viewID) : view_(viewID) {}
  // the state of a sequence (created on first use as CreateState(view, last
  // committed sequence), like createStateForNewConsensus, node.go:277-296)
  State& Open(int64_t sequenceID);
  State* Find(int64_t sequenceID);
  void Erase(int64_t sequenceID) { states_.erase(sequenceID); }
  size_t Size() const { return states_.size(); }
  int64_t LastCommitted() const { return last_committed_; }

  struct FlushOutcome {
    std::vector<bool> accepted;       // per snapshot vote: signature + verifyMsg passed
    std::vector<bool> applied;        // stored in its state (accepted, and the state had not advanced)
    std::vector<std::string> errors;  // the reference's error for each rejected vote
    std::vector<VoteMsg> commits;     // prepare flush: the commit vote of every sequence that became prepared
    std::vector<std::pair<ReplyMsg, RequestMsg>> replies;  // commit flush: every sequence that committed
  };
  FlushOutcome FlushPrepares(Crypto& c, const KeyTable& keys, const std::vector<VoteMsg>& snapshot);
  FlushOutcome FlushCommits(Crypto& c, const KeyTable& keys, const std::vector<VoteMsg>& snapshot);

 private:
  FlushOutcome flush(Crypto& c, const KeyTable& keys, const std::vector<VoteMsg>& snap, bool commit);
  int64_t view_;
  int64_t last_committed_ = -1;
  std::map<int64_t, State> states_;
};

// ---- pool/*.go --------------------------------------------------------
// Thread-safe map keyed as in the reference (RWMutex -> shared_mutex).
// GetAll returns a value-copy snapshot (Go map iteration order is random;
// here the order is by key -- no caller depends on it).
template <class T>
class MsgPool {
 public:
  using KeyFn = std::string (*)(const T&);
  explicit MsgPool(KeyFn key) : key_(key) {}
  void Add(const T& m) {
    std::unique_lock<std::shared_mutex> lk(mu_);
    pool_[key_(m)] = m;
  }
  void Del(const std::string& k) {
    std::unique_lock<std::shared_mutex> lk(mu_);
    pool_.erase(k);
  }
  void DelAll() {
    std::unique_lock<std::shared_mutex> lk(mu_);
    pool_.clear();
  }
  int MsgNum() const {
    std::shared_lock<std::shared_mutex> lk(mu_);
    return (int)pool_.size();
  }
  std::optional<T> Get(const std::string& k) const {
    std::shared_lock<std::shared_mutex> lk(mu_);
    auto it = pool_.find(k);
    if (it == pool_.end()) return std::nullopt;
    return it->second;
  }
  std::vector<T> GetAll() const {
    std::shared_lock<std::shared_mutex> lk(mu_);
    std::vector<T> out;
    out.reserve(pool_.size());
    for (auto& kv : pool_) out.push_back(kv.second);
    return out;
  }

 private:
  KeyFn key_;
  mutable std::shared_mutex mu_;
  std::map<std::string, T> pool_;
};

// requestPool.go:10 (ClientID), prepreparePool.go:9 (Digest), preparePool.go:9 /
// commitPool.go:9 / replyPool.go:9 (NodeID)
struct RequestMsgPool : MsgPool<RequestMsg> {
  RequestMsgPool() : MsgPool([](const RequestMsg& m) { return m.ClientID; }) {}
};
struct PrePrepareMsgPool : MsgPool<PrePrepareMsg> {
  PrePrepareMsgPool() : MsgPool([](const PrePrepareMsg& m) { return m.Digest; }) {}
};
struct PrepareMsgPool : MsgPool<VoteMsg> {
  PrepareMsgPool() : MsgPool([](const VoteMsg& m) { return m.NodeID; }) {}
};
struct CommitMsgPool : MsgPool<VoteMsg> {
  CommitMsgPool() : MsgPool([](const VoteMsg& m) { return m.NodeID; }) {}
};
struct ReplyMsgPool : MsgPool<ReplyMsg> {
  ReplyMsgPool() : MsgPool([](const ReplyMsg& m) { return m.NodeID; }) {}
};

// sequence-keyed vote pool (ConsensusTable's input): key = "<sequenceID>/<NodeID>",
// so votes of many sequences coexist and a re-sent vote overwrites its own entry
struct SeqVotePool : MsgPool<VoteMsg> {
  SeqVotePool() : MsgPool([](const VoteMsg& m) { return std::to_string(m.SequenceID) + "/" + m.NodeID; }) {}
};

}  // namespace pbft
