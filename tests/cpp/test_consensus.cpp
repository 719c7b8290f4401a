// test_consensus.cpp -- TEST PROGRAM for the C++ host mirror (simple_pbft_amd/csrc/host/pbft.h).
//
//   ./test_consensus oracle   -- CPU: crypto backend = the oracle (test double)
//   ./test_consensus gpu      -- MI355X: crypto backend = GpuCrypto (the product)
//
// Replays the reference's logged run (log/node1.log: 4 nodes MainNode,
// ReplicaNode1..3, view 10000000000, client1..3 with their logged timestamps and
// sequence IDs) through State / pools exactly as pbft/network/node.go drives
// them (GetReq :150, GetPrePrepare :179, GetPrepare :207, GetCommit :229,
// resolveReplyMsg :601), with the build-added signatures, flushing every
// pool snapshot through the batch verifier.  Also checks the reference's
// quorum and error semantics under corrupted / foreign votes, and the pools.
#include <array>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../oracle/oracle.h"
#include "pbft.h"

using namespace pbft;

static int g_fail = 0, g_pass = 0;
#define CHECK(c)                                                              \
  do {                                                                        \
    if (c) ++g_pass;                                                          \
    else {                                                                    \
      ++g_fail;                                                               \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
    }                                                                         \
  } while (0)

// ---------------------------------------------------------------- oracle-backed crypto (test double)
class OracleCrypto : public Crypto {
 public:
  std::vector<Digest32> Sha256(const std::vector<std::vector<uint8_t>>& msgs) override {
    std::vector<Digest32> out(msgs.size());
    for (size_t i = 0; i < msgs.size(); ++i) oracle_sha256(msgs[i].data(), msgs[i].size(), out[i].data());
    return out;
  }
  std::vector<bool> Verify(const std::vector<Digest32>& h, const std::vector<Sig>& s,
                           const std::vector<uint32_t>& k) override {
    std::vector<bool> out(h.size());
    for (size_t i = 0; i < h.size(); ++i)
      out[i] = k[i] < keys_.size() && oracle_ecdsa_p256_verify(h[i].data(), s[i].data(), keys_[k[i]].data()) == 1;
    return out;
  }
  void RegisterKeys(const std::vector<std::array<uint8_t, 64>>& pub) override { keys_ = pub; }

 private:
  std::vector<std::array<uint8_t, 64>> keys_;
};

// ---------------------------------------------------------------- signing (test infrastructure)
struct Signer {
  std::array<uint8_t, 32> d{};
  uint64_t nonce = 1;
  Sig sign(const Digest32& h) {
    Sig s{};
    for (;;) {
      std::array<uint8_t, 32> k{};
      for (int i = 0; i < 8; ++i) k[31 - i] = (uint8_t)((nonce * 0x9E3779B97F4A7C15ull) >> (8 * i));
      k[0] = d[0] ^ 0x5A;
      ++nonce;
      if (oracle_ecdsa_p256_sign(h.data(), d.data(), k.data(), s.data())) return s;
    }
  }
};

static Digest32 sha(const std::vector<uint8_t>& m) {
  Digest32 d;
  oracle_sha256(m.data(), m.size(), d.data());
  return d;
}

// ---------------------------------------------------------------- a node, as node.go drives State
constexpr int64_t kView = 10000000000;  // node.go:55

struct Node {
  std::string id;
  Signer key;
  std::unique_ptr<State> st;
  PrePrepareMsgPool pp_pool;
  PrepareMsgPool prep_pool;
  CommitMsgPool commit_pool;
  ReplyMsgPool reply_pool;
  std::vector<RequestMsg> committed;
  bool primary = false;

  void ensure_state() {  // createStateForNewConsensus (node.go:277-296)
    if (st) return;
    const int64_t last = committed.empty() ? -1 : committed.back().SequenceID;
    st = std::make_unique<State>(State::CreateState(kView, last));
  }
};

static std::vector<std::string> kNames = {"MainNode", "ReplicaNode1", "ReplicaNode2", "ReplicaNode3"};

struct Cluster {
  Crypto& c;
  KeyTable keys;
  std::vector<Node> nodes;
  std::vector<Signer> clients;

  explicit Cluster(Crypto& cr) : c(cr), nodes(4) {
    std::vector<std::array<uint8_t, 64>> pub;
    for (int i = 0; i < 4 + 3; ++i) {
      Signer s;
      s.d[31] = (uint8_t)(i + 1);
      s.d[0] = 0x11 * (i + 1);
      std::array<uint8_t, 64> xy{};
      oracle_p256_pubkey(s.d.data(), xy.data());
      pub.push_back(xy);
      if (i < 4) {
        nodes[i].id = kNames[i];
        nodes[i].key = s;
        keys.Add(kNames[i], i);
      } else {
        clients.push_back(s);
        keys.Add("client" + std::to_string(i - 3), i);
      }
    }
    nodes[0].primary = true;
    c.RegisterKeys(pub);
  }

  template <class M>
  void sign(M& m, Signer& s) {
    m.Signature = s.sign(sha(Marshal(m)));
  }
};

// one request through the whole protocol; returns the primary's valid reply count
static int run_request(Cluster& cl, RequestMsg req, int64_t now_ns, bool corrupt_commit_of_rn3,
                       const std::string& want_digest) {
  Crypto& c = cl.c;
  Node& P = cl.nodes[0];
  // client signs the request as sent (SequenceID 0, client.go:16-27)
  RequestMsg sent = req;
  sent.SequenceID = 0;
  const int ci = std::stoi(req.ClientID.substr(6)) - 1;
  cl.sign(sent, cl.clients[ci]);
  req.Signature = sent.Signature;
  CHECK(VerifySignatures(c, cl.keys, std::vector<RequestMsg>{req})[0]);

  // GetReq (node.go:150-174)
  P.ensure_state();
  auto ppr = P.st->StartConsensus(c, req, now_ns);
  CHECK(ppr.err.empty() && ppr.value);
  PrePrepareMsg pp = *ppr.value;
  CHECK(pp.Digest == want_digest);
  CHECK(pp.SequenceID == now_ns);
  pp.NodeID = P.id;
  cl.sign(pp, P.key);
  for (int r = 1; r < 4; ++r) cl.nodes[r].pp_pool.Add(pp);

  // replicas: GetPrePrepare (node.go:179-204), pre-prepare pool flushed as one batch
  std::vector<VoteMsg> prepares;
  for (int r = 1; r < 4; ++r) {
    Node& R = cl.nodes[r];
    auto snap = R.pp_pool.GetAll();
    auto sig_ok = VerifySignatures(c, cl.keys, snap);
    CHECK(sig_ok.size() == 1 && sig_ok[0]);
    R.ensure_state();
    auto pv = R.st->PrePrepare(c, snap[0]);
    CHECK(pv.err.empty() && pv.value);
    VoteMsg v = *pv.value;
    v.NodeID = R.id;
    cl.sign(v, R.key);
    prepares.push_back(v);
    R.pp_pool.Del(pp.Digest);
    CHECK(R.st->CurrentStage == Stage::PrePrepared);
  }
  for (auto& v : prepares)
    for (auto& n : cl.nodes)
      if (n.id != v.NodeID) n.prep_pool.Add(v);

  // every node: GetPrepare over its prepare snapshot (node.go:395-406, 559-577)
  std::vector<VoteMsg> commits;
  for (auto& n : cl.nodes) {
    auto snap = n.prep_pool.GetAll();
    CHECK((int)snap.size() >= 2 * f);
    BatchOutcome o;
    auto cv = n.st->PrepareBatch(c, cl.keys, snap, &o);
    CHECK(cv.err.empty() && cv.value);
    CHECK(n.st->CurrentStage == Stage::Prepared);
    VoteMsg v = *cv.value;
    v.NodeID = n.id;
    cl.sign(v, n.key);
    if (corrupt_commit_of_rn3 && n.id == "ReplicaNode3") v.Signature[40] ^= 0x01;
    commits.push_back(v);
    n.prep_pool.DelAll();
  }
  for (auto& v : commits)
    for (auto& n : cl.nodes)
      if (n.id != v.NodeID) n.commit_pool.Add(v);

  // every node: GetCommit over its commit snapshot (node.go:408-420, 580-598)
  for (auto& n : cl.nodes) {
    auto snap = n.commit_pool.GetAll();
    BatchOutcome o;
    auto rr = n.st->CommitBatch(c, cl.keys, snap, &o);
    CHECK(rr.err.empty() && rr.value);
    if (corrupt_commit_of_rn3 && n.id != "ReplicaNode3") {
      bool saw_bad = false;
      for (size_t i = 0; i < snap.size(); ++i)
        if (snap[i].NodeID == "ReplicaNode3") {
          // the bad vote is rejected unless the quorum was reached before it was applied
          if (i < o.applied) {
            CHECK(!o.accepted[i]);
            CHECK(o.errors[i] == "commit message signature is invalid");
          }
          saw_bad = true;
        }
      CHECK(saw_bad);
    }
    if (!rr.value) continue;
    CHECK(n.st->CurrentStage == Stage::Committed);
    CHECK(n.st->LastSequenceID == now_ns);
    ReplyMsg reply = rr.value->first;
    reply.NodeID = n.id;
    cl.sign(reply, n.key);
    n.committed.push_back(rr.value->second);
    // node.go:247-250: clear the logs; replicas go back to Idle (:258-261)
    n.st->MsgLogs_.ReqMsg.reset();
    n.st->MsgLogs_.PrepareMsgs.clear();
    n.st->MsgLogs_.CommitMsgs.clear();
    if (!n.primary) n.st->CurrentStage = Stage::Idle;
    n.commit_pool.DelAll();
    P.reply_pool.Add(reply);  // node.Reply -> primary's /reply (node.go:132-147)
  }

  // primary: resolveReplyMsg (node.go:422-431, 601-615) once >= f+1 replies
  auto replies = P.reply_pool.GetAll();
  CHECK((int)replies.size() >= f + 1);
  auto ok = VerifySignatures(c, cl.keys, replies);
  int good = 0;
  for (size_t i = 0; i < replies.size(); ++i) {
    good += ok[i];
    CHECK(replies[i].Result == "Executed" && replies[i].ClientID == req.ClientID &&
          replies[i].Timestamp == req.Timestamp && replies[i].ViewID == kView);
  }
  P.reply_pool.DelAll();
  P.st->CurrentStage = Stage::Idle;
  return good;
}

static void test_logged_run(Crypto& c) {
  Cluster cl(c);
  struct L { int64_t ts; const char* cid; int64_t seq; const char* dg; };
  // log/node1.log:3,20 / 30,49 / 59,80 (sequence IDs also in log/node2.log:22,43)
  const L logged[3] = {{1668519246, "client1", 1668519247222762700, "a63fc9e814525ac811f0ee3adcbe17bc46a58b828b8e1e07aa214f839f7365a9"},
                       {1668519366, "client2", 1668519366935576000, "e5485d99d877dc5b37daf4a69c51f3b8c6501b5ffcce86ca77d5a80f365c13e4"},
                       {1668519455, "client3", 1668519456530528400, "982077e48ed4e9a84ee74d5d35f4666e7fb5196169c8f75df1ca031d0563179a"}};
  for (int i = 0; i < 3; ++i) {
    RequestMsg r;
    r.Timestamp = logged[i].ts;
    r.ClientID = logged[i].cid;
    r.Operation = "printf";
    // request 2: ReplicaNode3's commit carries a flipped signature bit; the
    // other three commits still reach 2f at every receiver, and all four
    // replies (signed separately) verify at the primary
    const int good = run_request(cl, r, logged[i].seq, /*corrupt=*/i == 1, logged[i].dg);
    CHECK(good == 4);
  }
  for (auto& n : cl.nodes) {
    CHECK(n.committed.size() == 3);
    if (n.committed.size() == 3)
      for (int i = 0; i < 3; ++i) CHECK(n.committed[i].SequenceID == logged[i].seq);
  }
}

static void test_verifymsg_semantics(Crypto& c) {
  Cluster cl(c);
  State s = State::CreateState(kView, 5);
  RequestMsg r;
  r.Timestamp = 1;
  r.ClientID = "client1";
  r.Operation = "op";
  auto pp = s.StartConsensus(c, r, 3);  // now (3) <= last (5): bumped to 6 (pbft_impl.go:60-64)
  CHECK(pp.value && pp.value->SequenceID == 6);
  const std::string d = pp.value->Digest;
  CHECK(s.verifyMsg(c, kView, 6, d));
  CHECK(!s.verifyMsg(c, kView + 1, 6, d));          // wrong view
  CHECK(!s.verifyMsg(c, kView, 5, d));              // last >= seq
  std::string up = d;
  for (auto& ch : up) ch = (char)toupper(ch);
  CHECK(!s.verifyMsg(c, kView, 6, up));             // Go string compare is exact
  CHECK(!s.verifyMsg(c, kView, 6, d + "0"));
  // Prepare / Commit error strings (pbft_impl.go:117,147) and 2f quorum (:212,:227)
  VoteMsg bad;
  bad.ViewID = kView + 1;
  bad.SequenceID = 6;
  bad.Digest = d;
  bad.NodeID = "ReplicaNode1";
  auto e = s.Prepare(c, bad);
  CHECK(!e.value && e.err == "prepare message is corrupted");
  VoteMsg v1 = bad, v2 = bad;
  v1.ViewID = v2.ViewID = kView;
  v2.NodeID = "ReplicaNode2";
  auto a = s.Prepare(c, v1);
  CHECK(a.err.empty() && !a.value && !s.prepared());
  auto b = s.Prepare(c, v2);
  CHECK(b.value && b.value->Type == CommitMsg && s.prepared() && s.CurrentStage == Stage::Prepared);
  auto ce = s.Commit(c, bad);
  CHECK(!ce.value && ce.err == "commit message is corrupted");
  // batch flush: unsigned / foreign votes rejected, valid ones stored, stops at quorum
  State t = State::CreateState(kView, -1);
  RequestMsg r2 = r;
  auto pp2 = t.StartConsensus(c, r2, 100);
  std::vector<VoteMsg> snap;
  for (int i = 1; i < 4; ++i) {
    VoteMsg v;
    v.ViewID = kView;
    v.SequenceID = 100;
    v.Digest = pp2.value->Digest;
    v.NodeID = kNames[i];
    cl.sign(v, cl.nodes[i].key);
    snap.push_back(v);
  }
  snap[0].Signature[3] ^= 0x80;          // bad signature
  VoteMsg ghost = snap[1];
  ghost.NodeID = "Mallory";              // no registered key
  snap.insert(snap.begin() + 1, ghost);
  BatchOutcome o;
  auto cv = t.PrepareBatch(c, cl.keys, snap, &o);
  CHECK(cv.value && t.CurrentStage == Stage::Prepared);
  CHECK(o.accepted.size() == 4 && !o.accepted[0] && !o.accepted[1] && o.accepted[2] && o.accepted[3]);
  CHECK(o.errors[0] == "prepare message signature is invalid" && o.errors[1] == "prepare message signature is invalid");
  CHECK(t.MsgLogs_.PrepareMsgs.size() == 2 && o.applied == 4);
}

static void test_pools() {
  PrepareMsgPool p;
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&p, t] {
      for (int i = 0; i < 200; ++i) {
        VoteMsg v;
        v.NodeID = "n" + std::to_string(t * 1000 + i % 50);  // re-adds overwrite by key (preparePool.go:24)
        v.SequenceID = i;
        p.Add(v);
      }
    });
  for (auto& t : th) t.join();
  CHECK(p.MsgNum() == 8 * 50);
  auto all = p.GetAll();
  CHECK(all.size() == 400);
  p.Del("n0");
  CHECK(p.MsgNum() == 399 && !p.Get("n0") && p.Get("n1"));
  p.Del("absent");  // no-op like the reference's guarded delete
  p.DelAll();
  CHECK(p.MsgNum() == 0 && p.GetAll().empty());
  RequestMsgPool rq;
  RequestMsg r;
  r.ClientID = "c";
  rq.Add(r);
  rq.Add(r);
  CHECK(rq.MsgNum() == 1);
}

// Sequence-keyed consensus: K sequences in flight at one replica, every prepare
// and commit of all of them in ONE flush each (ConsensusTable), against the
// reference's one-state-at-a-time flush (State::PrepareBatch / CommitBatch) run
// per sequence over the same votes in the same order.
static void test_concurrent_sequences(Crypto& c) {
  Cluster cl(c);
  const int K = 40;
  const int64_t seq0 = 1668519247222762700;
  ConsensusTable tab(kView);
  std::vector<State> ref;
  std::vector<std::string> dg(K);
  for (int k = 0; k < K; ++k) {
    RequestMsg r;
    r.Timestamp = 1668519246 + k;
    r.ClientID = "client" + std::to_string(k % 3 + 1);
    r.Operation = k % 4 ? "printf" : "a<b>&\"c\"\n";  // HTML / escapes in the preimage
    RequestMsg r2 = r;
    auto pp = tab.Open(seq0 + k).StartConsensus(c, r, seq0 + k);
    ref.push_back(State::CreateState(kView, -1));
    auto pr = ref.back().StartConsensus(c, r2, seq0 + k);
    CHECK(pp.value && pr.value && pp.value->SequenceID == seq0 + k && pp.value->Digest == pr.value->Digest);
    dg[k] = pp.value->Digest;
  }
  CHECK(tab.Size() == (size_t)K);
  // prepares from ReplicaNode1..3 for every sequence, with faults:
  //   k % 5 == 1: ReplicaNode1's signature flipped;  k % 7 == 2: ReplicaNode2 votes an upper-case digest;
  //   k % 6 == 3: ReplicaNode3 votes the wrong view; k % 9 == 4: ReplicaNode1 AND ReplicaNode2 bad (no quorum)
  SeqVotePool pool;
  for (int k = 0; k < K; ++k)
    for (int r = 1; r < 4; ++r) {
      VoteMsg v;
      v.ViewID = kView;
      v.SequenceID = seq0 + k;
      v.Digest = dg[k];
      v.NodeID = kNames[r];
      v.Type = PrepareMsg;
      if (r == 2 && (k % 7 == 2 || k % 9 == 4))
        for (auto& ch : v.Digest) ch = (char)toupper(ch);
      if (r == 3 && k % 6 == 3) v.ViewID = kView + 1;
      cl.sign(v, cl.nodes[r].key);
      if (r == 1 && (k % 5 == 1 || k % 9 == 4)) v.Signature[7] ^= 0x10;
      pool.Add(v);
    }
  VoteMsg stray;  // a vote for a sequence this replica has no state for
  stray.ViewID = kView;
  stray.SequenceID = seq0 - 1;
  stray.Digest = dg[0];
  stray.NodeID = kNames[1];
  cl.sign(stray, cl.nodes[1].key);
  pool.Add(stray);
  const auto snap = pool.GetAll();
  CHECK(snap.size() == (size_t)(3 * K + 1));
  auto o = tab.FlushPrepares(c, cl.keys, snap);
  CHECK(o.accepted.size() == snap.size());
  int prepared = 0;
  for (int k = 0; k < K; ++k) {
    std::vector<VoteMsg> sub;
    std::vector<size_t> where;
    for (size_t i = 0; i < snap.size(); ++i)
      if (snap[i].SequenceID == seq0 + k) {
        sub.push_back(snap[i]);
        where.push_back(i);
      }
    BatchOutcome ro;
    auto cv = ref[k].PrepareBatch(c, cl.keys, sub, &ro);
    for (size_t j = 0; j < sub.size(); ++j) {
      CHECK(o.accepted[where[j]] == ro.accepted[j]);
      CHECK(o.errors[where[j]] == ro.errors[j]);
    }
    State* s = tab.Find(seq0 + k);
    CHECK(s && s->CurrentStage == ref[k].CurrentStage);
    CHECK(s && s->MsgLogs_.PrepareMsgs.size() == ref[k].MsgLogs_.PrepareMsgs.size());
    const bool want = !(k % 9 == 4) && !((k % 5 == 1) + (k % 7 == 2) + (k % 6 == 3) >= 2);
    CHECK((ref[k].CurrentStage == Stage::Prepared) == want);
    prepared += cv.value.has_value();
  }
  for (size_t i = 0; i < snap.size(); ++i)
    if (snap[i].SequenceID == seq0 - 1) CHECK(!o.accepted[i] && o.errors[i] == "prepare message is corrupted");
  CHECK((int)o.commits.size() == prepared && prepared > K / 2 && prepared < K);
  // commits from all four nodes for the prepared sequences; MainNode's commit bad on k % 4 == 0
  SeqVotePool cpool;
  for (const auto& cv : o.commits)
    for (int r = 0; r < 4; ++r) {
      VoteMsg v = cv;
      v.NodeID = kNames[r];
      cl.sign(v, cl.nodes[r].key);
      if (r == 0 && (v.SequenceID - seq0) % 4 == 0) v.Signature[20] ^= 0x01;
      cpool.Add(v);
    }
  const auto csnap = cpool.GetAll();
  auto co = tab.FlushCommits(c, cl.keys, csnap);
  CHECK((int)co.replies.size() == prepared);
  int64_t last = -1;
  for (int k = 0; k < K; ++k) {
    if (ref[k].CurrentStage != Stage::Prepared) continue;
    std::vector<VoteMsg> sub;
    for (const auto& v : csnap)
      if (v.SequenceID == seq0 + k) sub.push_back(v);
    auto rr = ref[k].CommitBatch(c, cl.keys, sub);
    State* s = tab.Find(seq0 + k);
    CHECK(rr.value && s && s->CurrentStage == Stage::Committed && ref[k].CurrentStage == Stage::Committed);
    CHECK(s && s->LastSequenceID == seq0 + k && s->MsgLogs_.CommitMsgs.size() == ref[k].MsgLogs_.CommitMsgs.size());
    last = seq0 + k;
  }
  CHECK(tab.LastCommitted() == last);
  // a state opened now starts after the highest committed sequence (createStateForNewConsensus)
  CHECK(tab.Open(seq0 + 1000).LastSequenceID == last);
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "oracle";
  std::unique_ptr<Crypto> c;
  if (mode == "gpu") {
    try {
      c = std::make_unique<GpuCrypto>();  // no CPU fallback: fails loudly without a GPU
    } catch (const std::exception& e) {
      std::fprintf(stderr, "GpuCrypto: %s\n", e.what());
      return 3;
    }
  } else {
    c = std::make_unique<OracleCrypto>();
  }
  test_pools();
  test_verifymsg_semantics(*c);
  test_logged_run(*c);
  test_concurrent_sequences(*c);
  std::printf("%s: %d checks passed, %d failed\n", mode.c_str(), g_pass, g_fail);
  return g_fail ? 1 : 0;
}
