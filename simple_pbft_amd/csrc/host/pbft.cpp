// pbft.cpp -- see pbft.h.  Reference line numbers refer to /root/reference.
#include "pbft.h"

#include <algorithm>
#include <climits>
#include <stdexcept>

#include "../../../include/pbftv.h"
#include "../gojson.h"

namespace pbft {

namespace {

const uint8_t* bytes(const std::string& s) { return reinterpret_cast<const uint8_t*>(s.data()); }

}  // namespace

// ---------------------------------------------------------------- preimages
std::vector<uint8_t> Marshal(const RequestMsg& m) {
  std::vector<uint8_t> out;
  pbftv::gojson::append_request(out, m.Timestamp, bytes(m.ClientID), m.ClientID.size(), bytes(m.Operation),
                                m.Operation.size(), m.SequenceID);
  return out;
}

std::vector<uint8_t> Marshal(const VoteMsg& m) {
  std::vector<uint8_t> out;
  pbftv::gojson::append_vote(out, m.ViewID, m.SequenceID, bytes(m.Digest), m.Digest.size(), bytes(m.NodeID),
                             m.NodeID.size(), (int64_t)m.Type);
  return out;
}

std::vector<uint8_t> Marshal(const ReplyMsg& m) {
  std::vector<uint8_t> out;
  pbftv::gojson::append_reply(out, m.ViewID, m.Timestamp, bytes(m.ClientID), m.ClientID.size(), bytes(m.NodeID),
                              m.NodeID.size(), bytes(m.Result), m.Result.size());
  return out;
}

std::vector<uint8_t> Marshal(const PrePrepareMsg& m) {
  std::vector<uint8_t> out;
  const RequestMsg empty;
  const RequestMsg& r = m.Request ? *m.Request : empty;
  pbftv::gojson::append_preprepare(out, m.ViewID, m.SequenceID, bytes(m.Digest), m.Digest.size(),
                                   m.Request.has_value(), r.Timestamp, bytes(r.ClientID), r.ClientID.size(),
                                   bytes(r.Operation), r.Operation.size(), r.SequenceID);
  return out;
}

// ---------------------------------------------------------------- GPU backend
GpuCrypto::GpuCrypto(uint32_t device_mask) {
  if (pbftv_open(&ctx_, device_mask) != PBFTV_OK) throw std::runtime_error(std::string("pbftv_open: ") + pbftv_last_error());
}

GpuCrypto::~GpuCrypto() { pbftv_close(ctx_); }

std::vector<Digest32> GpuCrypto::Sha256(const std::vector<std::vector<uint8_t>>& msgs) {
  const uint64_t n = msgs.size();
  std::vector<uint8_t> blob;
  std::vector<uint64_t> off(n);
  std::vector<uint32_t> len(n);
  for (uint64_t i = 0; i < n; ++i) {
    off[i] = blob.size();
    len[i] = (uint32_t)msgs[i].size();
    blob.insert(blob.end(), msgs[i].begin(), msgs[i].end());
  }
  blob.push_back(0);
  std::vector<Digest32> out(n);
  if (n && pbftv_sha256_batch(ctx_, blob.data(), off.data(), len.data(), n, out[0].data()) != PBFTV_OK)
    throw std::runtime_error(std::string("pbftv_sha256_batch: ") + pbftv_last_error());
  return out;
}

std::vector<bool> GpuCrypto::Verify(const std::vector<Digest32>& hashes, const std::vector<Sig>& sigs,
                                    const std::vector<uint32_t>& key_idx) {
  const uint64_t n = hashes.size();
  std::vector<uint8_t> bm((n + 7) / 8 + 1, 0);
  if (n && pbftv_ecdsa_p256_verify_batch(ctx_, hashes[0].data(), sigs[0].data(), key_idx.data(), n, bm.data()) !=
               PBFTV_OK)
    throw std::runtime_error(std::string("pbftv_ecdsa_p256_verify_batch: ") + pbftv_last_error());
  std::vector<bool> out(n);
  for (uint64_t i = 0; i < n; ++i) out[i] = (bm[i / 8] >> (i % 8)) & 1;
  return out;
}

// one pbftv_flush_votes call: the votes' fields column-wise, Go-JSON + SHA-256 +
// verifyMsg + ECDSA on the device
void GpuCrypto::FlushVotes(const std::vector<VoteMsg>& votes, const std::vector<uint32_t>& key_idx,
                           const std::vector<StateRef>& states, const std::vector<uint32_t>& state_idx,
                           std::vector<bool>& sig_ok, std::vector<bool>& msg_ok) {
  const uint64_t n = votes.size();
  sig_ok.assign(n, false);
  msg_ok.assign(n, false);
  if (n == 0) return;
  std::vector<int64_t> view(n), seq(n), type(n);
  std::vector<uint8_t> dblob, nblob;
  std::vector<uint64_t> doff(n), noff(n);
  std::vector<uint32_t> dlen(n), nlen(n);
  std::vector<Sig> sigs(n);
  for (uint64_t i = 0; i < n; ++i) {
    const VoteMsg& v = votes[i];
    view[i] = v.ViewID;
    seq[i] = v.SequenceID;
    type[i] = v.Type;
    doff[i] = dblob.size();
    dlen[i] = (uint32_t)v.Digest.size();
    dblob.insert(dblob.end(), v.Digest.begin(), v.Digest.end());
    noff[i] = nblob.size();
    nlen[i] = (uint32_t)v.NodeID.size();
    nblob.insert(nblob.end(), v.NodeID.begin(), v.NodeID.end());
    sigs[i] = v.Signature;
  }
  dblob.push_back(0);
  nblob.push_back(0);
  const uint32_t k = (uint32_t)states.size();
  std::vector<int64_t> sv(k + 1), sl(k + 1);
  std::vector<uint8_t> sd(32 * (k + 1));
  for (uint32_t s = 0; s < k; ++s) {
    sv[s] = states[s].view;
    sl[s] = states[s].last_seq;
    std::copy(states[s].req_digest.begin(), states[s].req_digest.end(), sd.begin() + 32 * s);
  }
  std::vector<uint8_t> sbm((n + 7) / 8 + 1), mbm((n + 7) / 8 + 1);
  if (pbftv_flush_votes(ctx_, n, view.data(), seq.data(), dblob.data(), doff.data(), dlen.data(), nblob.data(),
                        noff.data(), nlen.data(), type.data(), sigs[0].data(), key_idx.data(), k, sv.data(), sl.data(),
                        sd.data(), state_idx.data(), nullptr, sbm.data(), mbm.data()) != PBFTV_OK)
    throw std::runtime_error(std::string("pbftv_flush_votes: ") + pbftv_last_error());
  for (uint64_t i = 0; i < n; ++i) {
    sig_ok[i] = (sbm[i / 8] >> (i % 8)) & 1;
    msg_ok[i] = (mbm[i / 8] >> (i % 8)) & 1;
  }
}

void GpuCrypto::RegisterKeys(const std::vector<std::array<uint8_t, 64>>& pub_xy) {
  if (pbftv_register_keys(ctx_, pub_xy.empty() ? nullptr : pub_xy[0].data(), (uint32_t)pub_xy.size(), nullptr) !=
      PBFTV_OK)
    throw std::runtime_error(std::string("pbftv_register_keys: ") + pbftv_last_error());
}

// ---------------------------------------------------------------- utils / digest
std::string ToHex(const Digest32& d) {
  static const char hx[] = "0123456789abcdef";  // encoding/hex: lowercase
  std::string s(64, '0');
  for (int i = 0; i < 32; ++i) {
    s[2 * i] = hx[d[i] >> 4];
    s[2 * i + 1] = hx[d[i] & 15];
  }
  return s;
}

std::string Hash(Crypto& c, const std::vector<uint8_t>& content) { return ToHex(c.Sha256({content})[0]); }

std::string digest(Crypto& c, const RequestMsg& r) { return Hash(c, Marshal(r)); }

// ---------------------------------------------------------------- signatures
template <class M>
static std::vector<bool> verify_sigs(Crypto& c, const KeyTable& keys, const std::vector<M>& msgs,
                                     std::string (*signer)(const M&), std::vector<uint8_t> (*preimage)(const M&)) {
  const size_t n = msgs.size();
  std::vector<std::vector<uint8_t>> pre(n);
  std::vector<Sig> sigs(n);
  std::vector<uint32_t> kidx(n, 0);
  std::vector<bool> known(n, false);
  for (size_t i = 0; i < n; ++i) {
    pre[i] = preimage(msgs[i]);
    sigs[i] = msgs[i].Signature;
    if (auto k = keys.Find(signer(msgs[i]))) {
      kidx[i] = *k;
      known[i] = true;
    }
  }
  if (n == 0) return {};
  std::vector<bool> ok = c.Verify(c.Sha256(pre), sigs, kidx);
  for (size_t i = 0; i < n; ++i) ok[i] = ok[i] && known[i];
  return ok;
}

std::vector<bool> VerifySignatures(Crypto& c, const KeyTable& keys, const std::vector<VoteMsg>& v) {
  return verify_sigs<VoteMsg>(c, keys, v, [](const VoteMsg& m) { return m.NodeID; },
                              [](const VoteMsg& m) { return Marshal(m); });
}

std::vector<bool> VerifySignatures(Crypto& c, const KeyTable& keys, const std::vector<ReplyMsg>& v) {
  return verify_sigs<ReplyMsg>(c, keys, v, [](const ReplyMsg& m) { return m.NodeID; },
                               [](const ReplyMsg& m) { return Marshal(m); });
}

std::vector<bool> VerifySignatures(Crypto& c, const KeyTable& keys, const std::vector<PrePrepareMsg>& v) {
  return verify_sigs<PrePrepareMsg>(c, keys, v, [](const PrePrepareMsg& m) { return m.NodeID; },
                                    [](const PrePrepareMsg& m) { return Marshal(m); });
}

// A client signs the request as it sends it, before the primary assigns the
// sequence ID (client.go:16-27 sends SequenceID 0).
std::vector<bool> VerifySignatures(Crypto& c, const KeyTable& keys, const std::vector<RequestMsg>& v) {
  return verify_sigs<RequestMsg>(c, keys, v, [](const RequestMsg& m) { return m.ClientID; },
                                 [](const RequestMsg& m) {
                                   RequestMsg sent = m;
                                   sent.SequenceID = 0;
                                   return Marshal(sent);
                                 });
}

// ---------------------------------------------------------------- State
State State::CreateState(int64_t viewID, int64_t lastSequenceID) {
  State s;
  s.ViewID = viewID;
  s.LastSequenceID = lastSequenceID;
  s.CurrentStage = Stage::Idle;
  return s;
}

const std::string& State::request_digest(Crypto& c) {
  if (!req_digest_) {
    // json.Marshal of a nil *RequestMsg is "null"
    req_digest_ = MsgLogs_.ReqMsg ? digest(c, *MsgLogs_.ReqMsg) : Hash(c, {'n', 'u', 'l', 'l'});
  }
  return *req_digest_;
}

Result<PrePrepareMsg> State::StartConsensus(Crypto& c, RequestMsg& request, int64_t now_unix_nano) {
  int64_t sequenceID = now_unix_nano;
  if (LastSequenceID != -1) {
    while (LastSequenceID >= sequenceID) sequenceID += 1;
  }
  request.SequenceID = sequenceID;
  MsgLogs_.ReqMsg = request;
  req_digest_.reset();
  const std::string d = request_digest(c);
  CurrentStage = Stage::PrePrepared;
  PrePrepareMsg pp;
  pp.ViewID = ViewID;
  pp.SequenceID = sequenceID;
  pp.Digest = d;
  pp.Request = request;
  return {pp, ""};
}

Result<VoteMsg> State::PrePrepare(Crypto& c, const PrePrepareMsg& pp) {
  MsgLogs_.ReqMsg = pp.Request;
  req_digest_.reset();
  if (!verifyMsg(c, pp.ViewID, pp.SequenceID, pp.Digest)) return {std::nullopt, "pre-prepare message is corrupted"};
  CurrentStage = Stage::PrePrepared;
  VoteMsg v;
  v.ViewID = ViewID;
  v.SequenceID = pp.SequenceID;
  v.Digest = pp.Digest;
  v.Type = PrepareMsg;
  return {v, ""};
}

Result<VoteMsg> State::Prepare(Crypto& c, const VoteMsg& m) {
  if (!verifyMsg(c, m.ViewID, m.SequenceID, m.Digest)) return {std::nullopt, "prepare message is corrupted"};
  MsgLogs_.PrepareMsgs[m.NodeID] = m;
  if (prepared()) {
    CurrentStage = Stage::Prepared;
    VoteMsg v;
    v.ViewID = ViewID;
    v.SequenceID = m.SequenceID;
    v.Digest = m.Digest;
    v.Type = CommitMsg;
    return {v, ""};
  }
  return {std::nullopt, ""};
}

Result<std::pair<ReplyMsg, RequestMsg>> State::Commit(Crypto& c, const VoteMsg& m) {
  if (!verifyMsg(c, m.ViewID, m.SequenceID, m.Digest)) return {std::nullopt, "commit message is corrupted"};
  MsgLogs_.CommitMsgs[m.NodeID] = m;
  if (committed()) {
    CurrentStage = Stage::Committed;
    LastSequenceID = m.SequenceID;
    ReplyMsg r;
    r.ViewID = ViewID;
    r.Timestamp = MsgLogs_.ReqMsg->Timestamp;
    r.ClientID = MsgLogs_.ReqMsg->ClientID;
    r.Result = "Executed";
    return {std::make_pair(r, *MsgLogs_.ReqMsg), ""};
  }
  return {std::nullopt, ""};
}

bool State::verifyMsg(Crypto& c, int64_t viewID, int64_t sequenceID, const std::string& digestGot) {
  if (ViewID != viewID) return false;                                  // pbft_impl.go:178
  if (LastSequenceID != -1 && LastSequenceID >= sequenceID) return false;  // :184-188
  return digestGot == request_digest(c);                              // :190-199, Go string compare
}

bool State::prepared() const {
  if (!MsgLogs_.ReqMsg) return false;
  return (int)MsgLogs_.PrepareMsgs.size() >= 2 * f;
}

bool State::committed() const {
  if (!prepared()) return false;
  return (int)MsgLogs_.CommitMsgs.size() >= 2 * f;
}

std::vector<bool> State::verify_votes(Crypto& c, const KeyTable& keys, const std::vector<VoteMsg>& snap,
                                      std::vector<std::string>& errs, const char* what) {
  std::vector<bool> sig_ok = VerifySignatures(c, keys, snap);  // one SHA-256 batch + one ECDSA batch
  std::vector<bool> ok(snap.size());
  errs.assign(snap.size(), "");
  for (size_t i = 0; i < snap.size(); ++i) {
    const bool msg_ok = verifyMsg(c, snap[i].ViewID, snap[i].SequenceID, snap[i].Digest);  // digest hashed once
    ok[i] = sig_ok[i] && msg_ok;
    if (!msg_ok) errs[i] = std::string(what) + " message is corrupted";
    else if (!sig_ok[i]) errs[i] = std::string(what) + " message signature is invalid";
  }
  return ok;
}

Result<VoteMsg> State::PrepareBatch(Crypto& c, const KeyTable& keys, const std::vector<VoteMsg>& snap,
                                    BatchOutcome* outcome) {
  BatchOutcome local;
  BatchOutcome& o = outcome ? *outcome : local;
  o.accepted = verify_votes(c, keys, snap, o.errors, "prepare");
  o.applied = 0;
  for (size_t i = 0; i < snap.size(); ++i) {
    o.applied = i + 1;
    if (!o.accepted[i]) continue;
    MsgLogs_.PrepareMsgs[snap[i].NodeID] = snap[i];
    if (prepared()) {  // MSGENOUGH: the reference stops taking this snapshot here (node.go:564-566)
      CurrentStage = Stage::Prepared;
      VoteMsg v;
      v.ViewID = ViewID;
      v.SequenceID = snap[i].SequenceID;
      v.Digest = snap[i].Digest;
      v.Type = CommitMsg;
      return {v, ""};
    }
  }
  return {std::nullopt, ""};
}

Result<std::pair<ReplyMsg, RequestMsg>> State::CommitBatch(Crypto& c, const KeyTable& keys,
                                                           const std::vector<VoteMsg>& snap, BatchOutcome* outcome) {
  BatchOutcome local;
  BatchOutcome& o = outcome ? *outcome : local;
  o.accepted = verify_votes(c, keys, snap, o.errors, "commit");
  o.applied = 0;
  for (size_t i = 0; i < snap.size(); ++i) {
    o.applied = i + 1;
    if (!o.accepted[i]) continue;
    MsgLogs_.CommitMsgs[snap[i].NodeID] = snap[i];
    if (committed()) {
      CurrentStage = Stage::Committed;
      LastSequenceID = snap[i].SequenceID;
      ReplyMsg r;
      r.ViewID = ViewID;
      r.Timestamp = MsgLogs_.ReqMsg->Timestamp;
      r.ClientID = MsgLogs_.ReqMsg->ClientID;
      r.Result = "Executed";
      return {std::make_pair(r, *MsgLogs_.ReqMsg), ""};
    }
  }
  return {std::nullopt, ""};
}

// ---------------------------------------------------------------- multi-state flush
void Crypto::FlushVotes(const std::vector<VoteMsg>& votes, const std::vector<uint32_t>& key_idx,
                        const std::vector<StateRef>& states, const std::vector<uint32_t>& state_idx,
                        std::vector<bool>& sig_ok, std::vector<bool>& msg_ok) {
  const size_t n = votes.size();
  std::vector<std::vector<uint8_t>> pre(n);
  std::vector<Sig> sigs(n);
  for (size_t i = 0; i < n; ++i) {
    pre[i] = Marshal(votes[i]);
    sigs[i] = votes[i].Signature;
  }
  sig_ok = n ? Verify(Sha256(pre), sigs, key_idx) : std::vector<bool>();
  msg_ok.assign(n, false);
  for (size_t i = 0; i < n; ++i) {
    if (state_idx[i] >= states.size()) continue;
    const StateRef& s = states[state_idx[i]];
    msg_ok[i] = votes[i].ViewID == s.view && (s.last_seq == -1 || s.last_seq < votes[i].SequenceID) &&
                votes[i].Digest == ToHex(s.req_digest);
  }
}

static Digest32 from_hex(const std::string& h) {
  Digest32 d{};
  auto nib = [](char c) { return (uint8_t)(c <= '9' ? c - '0' : c - 'a' + 10); };
  for (int i = 0; i < 32 && 2 * i + 1 < (int)h.size(); ++i) d[i] = (uint8_t)(nib(h[2 * i]) << 4 | nib(h[2 * i + 1]));
  return d;
}

State& ConsensusTable::Open(int64_t sequenceID) {
  auto it = states_.find(sequenceID);
  if (it == states_.end()) it = states_.emplace(sequenceID, State::CreateState(view_, last_committed_)).first;
  return it->second;
}

State* ConsensusTable::Find(int64_t sequenceID) {
  auto it = states_.find(sequenceID);
  return it == states_.end() ? nullptr : &it->second;
}

ConsensusTable::FlushOutcome ConsensusTable::FlushPrepares(Crypto& c, const KeyTable& keys,
                                                           const std::vector<VoteMsg>& snapshot) {
  return flush(c, keys, snapshot, false);
}

ConsensusTable::FlushOutcome ConsensusTable::FlushCommits(Crypto& c, const KeyTable& keys,
                                                          const std::vector<VoteMsg>& snapshot) {
  return flush(c, keys, snapshot, true);
}

ConsensusTable::FlushOutcome ConsensusTable::flush(Crypto& c, const KeyTable& keys, const std::vector<VoteMsg>& snap,
                                                   bool commit) {
  const size_t n = snap.size();
  FlushOutcome o;
  o.accepted.assign(n, false);
  o.applied.assign(n, false);
  o.errors.assign(n, "");
  // route every vote to its sequence's state; each state's request is hashed once
  std::map<int64_t, uint32_t> ref_of;
  std::vector<Crypto::StateRef> refs;
  std::vector<uint32_t> st_idx(n, UINT32_MAX), kidx(n, 0);
  std::vector<bool> known(n, false);
  for (size_t i = 0; i < n; ++i) {
    auto it = states_.find(snap[i].SequenceID);
    if (it != states_.end()) {
      auto ins = ref_of.emplace(it->first, (uint32_t)refs.size());
      if (ins.second) {
        State& s = it->second;
        refs.push_back({s.ViewID, s.LastSequenceID, from_hex(s.request_digest(c))});
      }
      st_idx[i] = ins.first->second;
    }
    if (auto k = keys.Find(snap[i].NodeID)) {
      kidx[i] = *k;
      known[i] = true;
    }
  }
  std::vector<bool> sig_ok, msg_ok;
  if (n) c.FlushVotes(snap, kidx, refs, st_idx, sig_ok, msg_ok);
  const std::string what = commit ? "commit" : "prepare";
  for (size_t i = 0; i < n; ++i) {
    const bool m = st_idx[i] != UINT32_MAX && msg_ok[i];
    const bool sg = known[i] && sig_ok[i];
    o.accepted[i] = m && sg;
    if (!m) o.errors[i] = what + " message is corrupted";  // pbft_impl.go:117,147
    else if (!sg) o.errors[i] = what + " message signature is invalid";
    if (!o.accepted[i]) continue;
    State& s = states_.at(snap[i].SequenceID);
    // only a state at this vote's stage takes it; once it advances it stops
    // taking this snapshot's votes (MSGENOUGH, node.go:564-566, 585-587)
    if (s.CurrentStage != (commit ? Stage::Prepared : Stage::PrePrepared)) continue;
    o.applied[i] = true;
    if (!commit) {
      s.MsgLogs_.PrepareMsgs[snap[i].NodeID] = snap[i];
      if (s.prepared()) {
        s.CurrentStage = Stage::Prepared;
        VoteMsg v;
        v.ViewID = s.ViewID;
        v.SequenceID = snap[i].SequenceID;
        v.Digest = snap[i].Digest;
        v.Type = CommitMsg;
        o.commits.push_back(v);
      }
    } else {
      s.MsgLogs_.CommitMsgs[snap[i].NodeID] = snap[i];
      if (s.committed()) {
        s.CurrentStage = Stage::Committed;
        s.LastSequenceID = snap[i].SequenceID;
        last_committed_ = std::max(last_committed_, snap[i].SequenceID);
        ReplyMsg r;
        r.ViewID = s.ViewID;
        r.Timestamp = s.MsgLogs_.ReqMsg->Timestamp;
        r.ClientID = s.MsgLogs_.ReqMsg->ClientID;
        r.Result = "Executed";
        o.replies.emplace_back(r, *s.MsgLogs_.ReqMsg);
      }
    }
  }
  return o;
}

}  // namespace pbft
