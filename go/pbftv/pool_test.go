package pbftv

// A pool flush checked against the reference's own code path run in Go:
// votes, pre-prepares, requests and replies are marshalled with
// encoding/json, signed with crypto/ecdsa (P-256, crypto/rand nonces), some
// corrupted (bad signature, wrong digest, wrong view, stale sequence ID), and
// every bit the library returns is compared with crypto/ecdsa.Verify and with
// verifyMsg below, which is pbft/consensus/pbft_impl.go:176-202 verbatim in
// behaviour.  Needs a GPU (skipped otherwise).

import (
	"crypto/ecdsa"
	"crypto/elliptic"
	"crypto/rand"
	"crypto/sha256"
	"encoding/hex"
	"encoding/json"
	"fmt"
	"math/big"
	mrand "math/rand"
	"testing"
)

// verifyMsg restates State.verifyMsg (pbft_impl.go:176-202): view, then the
// sequence ID against the last committed one, then the digest string of the
// state's request (digest(), :235-243) compared with Go's string equality.
func verifyMsg(stView, stLast int64, req *RequestMsg, viewID, seqID int64, digestGot string) bool {
	if stView != viewID {
		return false
	}
	if stLast != -1 && stLast >= seqID {
		return false
	}
	pre, err := json.Marshal(req)
	if err != nil {
		return false
	}
	h := sha256.Sum256(pre)
	return digestGot == hex.EncodeToString(h[:])
}

type signer struct {
	keys []*ecdsa.PrivateKey
	raw  [][64]byte
}

func newSigner(t *testing.T, n int) *signer {
	s := &signer{}
	for i := 0; i < n; i++ {
		k, err := ecdsa.GenerateKey(elliptic.P256(), rand.Reader)
		if err != nil {
			t.Fatal(err)
		}
		var r [64]byte
		k.PublicKey.X.FillBytes(r[:32])
		k.PublicKey.Y.FillBytes(r[32:])
		s.keys, s.raw = append(s.keys, k), append(s.raw, r)
	}
	return s
}

// sign returns r||s over SHA-256(json.Marshal(msg)) and that hash.
func (s *signer) sign(t *testing.T, key int, msg interface{}) ([64]byte, [32]byte) {
	pre, err := json.Marshal(msg)
	if err != nil {
		t.Fatal(err)
	}
	h := sha256.Sum256(pre)
	r, ss, err := ecdsa.Sign(rand.Reader, s.keys[key], h[:])
	if err != nil {
		t.Fatal(err)
	}
	var out [64]byte
	r.FillBytes(out[:32])
	ss.FillBytes(out[32:])
	return out, h
}

func (s *signer) verify(key int, h [32]byte, sig [64]byte) bool {
	return ecdsa.Verify(&s.keys[key].PublicKey, h[:], new(big.Int).SetBytes(sig[:32]), new(big.Int).SetBytes(sig[32:]))
}

func TestFlushVotesAgainstGo(t *testing.T) {
	x := gpu(t)
	s := newSigner(t, 4)
	if _, err := x.RegisterKeys(s.raw); err != nil {
		t.Fatal(err)
	}
	rng := mrand.New(mrand.NewSource(7))
	const nStates = 5
	reqs := make([]*RequestMsg, nStates)
	states := make([]State, nStates)
	for i := range reqs {
		reqs[i] = &RequestMsg{Timestamp: int64(1668519246 + i), ClientID: fmt.Sprintf("client%d", i),
			Operation: "printf", SequenceID: int64(1668519247222762700 + 1000*i)}
		pre, _ := json.Marshal(reqs[i])
		states[i] = State{ViewID: 10000000000, LastSequenceID: -1, ReqDigest: sha256.Sum256(pre)}
		if i > 0 {
			states[i].LastSequenceID = reqs[i-1].SequenceID
		}
	}
	var votes []VoteMsg
	var sigs [][64]byte
	var keys, stIdx []uint32
	var wantSig, wantMsg []bool
	for i := 0; i < 700; i++ {
		st := rng.Intn(nStates)
		dg := hex.EncodeToString(states[st].ReqDigest[:])
		v := VoteMsg{ViewID: 10000000000, SequenceID: reqs[st].SequenceID, Digest: dg,
			NodeID: fmt.Sprintf("ReplicaNode%d", i%4), MsgType: MsgType(i % 2)}
		switch rng.Intn(8) {
		case 1:
			v.Digest = dg[:63] + "0" // wrong digest
		case 2:
			v.ViewID++ // wrong view
		case 3:
			if st > 0 {
				v.SequenceID = reqs[st-1].SequenceID // stale: already committed
			}
		case 4:
			v.Digest = fmt.Sprintf("%X", states[st].ReqDigest[:]) // upper case: Go's string compare rejects it
		}
		key := rng.Intn(4)
		sig, h := s.sign(t, key, &v)
		if rng.Intn(8) == 0 {
			sig[rng.Intn(64)] ^= 1 << uint(rng.Intn(8))
		}
		votes, sigs, keys = append(votes, v), append(sigs, sig), append(keys, uint32(key))
		stIdx = append(stIdx, uint32(st))
		wantSig = append(wantSig, s.verify(key, h, sig))
		wantMsg = append(wantMsg, verifyMsg(states[st].ViewID, states[st].LastSequenceID, reqs[st], v.ViewID,
			v.SequenceID, v.Digest))
	}
	res, err := x.FlushVotes(votes, sigs, keys, states, stIdx)
	if err != nil {
		t.Fatal(err)
	}
	nBadSig, nBadMsg := 0, 0
	for i, v := range votes {
		pre, _ := json.Marshal(&v)
		if res.Digests[i] != sha256.Sum256(pre) {
			t.Errorf("vote %d: digest of the Go-JSON preimage differs", i)
		}
		if res.SigOK[i] != wantSig[i] {
			t.Errorf("vote %d: library sig %v, crypto/ecdsa %v", i, res.SigOK[i], wantSig[i])
		}
		if res.MsgOK[i] != wantMsg[i] {
			t.Errorf("vote %d: library verifyMsg %v, Go %v", i, res.MsgOK[i], wantMsg[i])
		}
		if !wantSig[i] {
			nBadSig++
		}
		if !wantMsg[i] {
			nBadMsg++
		}
	}
	if nBadSig == 0 || nBadMsg == 0 {
		t.Fatalf("no corrupted votes (%d bad signatures, %d bad messages)", nBadSig, nBadMsg)
	}
}

func TestFlushRequestsRepliesPrePreparesAgainstGo(t *testing.T) {
	x := gpu(t)
	s := newSigner(t, 5) // 4 nodes + the client (key 4)
	if _, err := x.RegisterKeys(s.raw); err != nil {
		t.Fatal(err)
	}
	const n = 300
	var reqs []RequestMsg
	var rsig [][64]byte
	var rkey []uint32
	var assigned []int64
	var wantReq []bool
	var pps []PrePrepareMsg
	var psig [][64]byte
	var pkey, pst []uint32
	var wantPP, wantPPMsg []bool
	var reps []ReplyMsg
	var ysig [][64]byte
	var ykey []uint32
	var wantRep []bool
	states := []State{{ViewID: 10000000000, LastSequenceID: -1}, {ViewID: 10000000000, LastSequenceID: 1668519247222762700}}
	for i := 0; i < n; i++ {
		q := RequestMsg{Timestamp: int64(1668519246 + i), ClientID: fmt.Sprintf("client%d", i), Operation: "printf"}
		sig, h := s.sign(t, 4, &q)
		if i%17 == 0 {
			sig[5] ^= 0x40
		}
		reqs, rsig, rkey = append(reqs, q), append(rsig, sig), append(rkey, 4)
		wantReq = append(wantReq, s.verify(4, h, sig))
		seq := int64(1668519247222762700 + 1000*(i%3))
		assigned = append(assigned, seq)

		q.SequenceID = seq
		pre, _ := json.Marshal(&q)
		d := sha256.Sum256(pre)
		p := PrePrepareMsg{ViewID: 10000000000, SequenceID: seq, Digest: hex.EncodeToString(d[:]), RequestMsg: &q}
		if i%11 == 0 {
			p.Digest = hex.EncodeToString(d[1:]) + "00"
		}
		if i%13 == 0 {
			p.RequestMsg = nil // digest() of a nil request is Hash("null")
		}
		st := i % 2
		sig, h = s.sign(t, 0, &p)
		if i%19 == 0 {
			sig[40] ^= 2
		}
		pps, psig, pkey, pst = append(pps, p), append(psig, sig), append(pkey, 0), append(pst, uint32(st))
		wantPP = append(wantPP, s.verify(0, h, sig))
		wantPPMsg = append(wantPPMsg, verifyMsg(states[st].ViewID, states[st].LastSequenceID, p.RequestMsg, p.ViewID,
			p.SequenceID, p.Digest))

		r := ReplyMsg{ViewID: 10000000000, Timestamp: q.Timestamp, ClientID: q.ClientID,
			NodeID: fmt.Sprintf("ReplicaNode%d", i%4), Result: "Executed"}
		node := i % 4
		sig, h = s.sign(t, node, &r)
		if i%23 == 0 {
			node = (node + 1) % 4 // the wrong replica's key
		}
		reps, ysig, ykey = append(reps, r), append(ysig, sig), append(ykey, uint32(node))
		wantRep = append(wantRep, s.verify(node, h, sig))
	}
	rq, err := x.FlushRequests(reqs, rsig, rkey, assigned)
	if err != nil {
		t.Fatal(err)
	}
	for i := range reqs {
		q := reqs[i]
		pre, _ := json.Marshal(&q)
		q.SequenceID = assigned[i]
		cpre, _ := json.Marshal(&q)
		if rq.SigOK[i] != wantReq[i] || rq.Digests[i] != sha256.Sum256(pre) ||
			rq.ConsensusDigests[i] != sha256.Sum256(cpre) {
			t.Errorf("request %d differs from Go", i)
		}
	}
	pr, err := x.FlushPrePrepares(pps, psig, pkey, states, pst)
	if err != nil {
		t.Fatal(err)
	}
	for i, p := range pps {
		pre, _ := json.Marshal(&p)
		rpre, _ := json.Marshal(p.RequestMsg)
		if pr.SigOK[i] != wantPP[i] || pr.MsgOK[i] != wantPPMsg[i] || pr.Digests[i] != sha256.Sum256(pre) ||
			pr.ReqDigests[i] != sha256.Sum256(rpre) {
			t.Errorf("pre-prepare %d differs from Go", i)
		}
	}
	_, ok, err := x.FlushReplies(reps, ysig, ykey)
	if err != nil {
		t.Fatal(err)
	}
	for i := range reps {
		if ok[i] != wantRep[i] {
			t.Errorf("reply %d: library %v, crypto/ecdsa %v", i, ok[i], wantRep[i])
		}
	}
}

// A quorum certificate both ways: 2f (the reference's prepared()/committed()
// count, pbft_impl.go:212,227) and 2f+1.
func TestQCVerify(t *testing.T) {
	x := gpu(t)
	s := newSigner(t, 4)
	if _, err := x.RegisterKeys(s.raw); err != nil {
		t.Fatal(err)
	}
	v := VoteMsg{ViewID: 10000000000, SequenceID: 1, Digest: "00", NodeID: "n", MsgType: CommitMsg}
	var hs [][32]byte
	var sigs [][64]byte
	for k := 1; k < 4; k++ {
		sig, h := s.sign(t, k, &v)
		hs, sigs = append(hs, h), append(sigs, sig)
	}
	keys := []uint32{1, 2, 3}
	_, acc, reached, err := x.QCVerify(hs, sigs, keys, 3)
	if err != nil || acc != 3 || !reached {
		t.Fatalf("valid QC: %d %v %v", acc, reached, err)
	}
	sigs[1][3] ^= 1
	_, acc, reached, _ = x.QCVerify(hs, sigs, keys, 3)
	if acc != 2 || reached {
		t.Fatalf("one bad vote, 2f+1: %d %v", acc, reached)
	}
	if _, _, reached, _ = x.QCVerify(hs, sigs, keys, 2); !reached {
		t.Fatal("one bad vote, 2f: quorum should hold")
	}
}
