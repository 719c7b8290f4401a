package pbftv

/*
#include "pbftv.h"
*/
import "C"

import "unsafe"

// Pool flushes (SURVEY.md §8 a8/a9, f3): one GPU round trip per pool
// snapshot instead of one verifyMsg per message.  Each flush builds the
// go1.19 json.Marshal preimages of the messages on the GPU, hashes them,
// verifies the signatures (sigs[i] = r||s over SHA-256 of the unsigned
// message, key keyIdx[i]) and applies State.verifyMsg
// (pbft/consensus/pbft_impl.go:176-202) where the reference does.  A message
// counts toward its state's quorum iff SigOK[i] && MsgOK[i].

// VoteResult is the outcome of FlushVotes.
type VoteResult struct {
	Digests [][32]byte // SHA-256(json.Marshal(vote)): the signed preimage's hash
	SigOK   []bool
	MsgOK   []bool // verifyMsg against states[stateIdx[i]] (false when the index is out of range)
}

func sigPtr(sigs [][64]byte) *C.uint8_t {
	if len(sigs) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&sigs[0]))
}

func digestPtr(d [][32]byte) *C.uint8_t {
	if len(d) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&d[0]))
}

func stateColumns(states []State) (view, last []int64, req [][32]byte) {
	view, last, req = make([]int64, len(states)+1), make([]int64, len(states)+1), make([][32]byte, len(states)+1)
	for i, s := range states {
		view[i], last[i], req[i] = s.ViewID, s.LastSequenceID, s.ReqDigest
	}
	return view, last, req
}

// FlushVotes replaces the per-vote loops of resolvePrepareMsg /
// resolveCommitMsg (pbft/network/node.go:559-598) for a GetAllPreMsg /
// GetAllCmMsg snapshot across any number of consensus states
// (pbftv_flush_votes).
func (x *Ctx) FlushVotes(votes []VoteMsg, sigs [][64]byte, keyIdx []uint32, states []State,
	stateIdx []uint32) (VoteResult, error) {
	n := len(votes)
	if n == 0 {
		return VoteResult{}, nil
	}
	if len(sigs) != n || len(keyIdx) != n || len(stateIdx) != n {
		return VoteResult{}, &Error{Code: EINVAL, Msg: "column lengths differ"}
	}
	views, seqs, types := make([]int64, n), make([]int64, n), make([]int64, n)
	dg, ids := make([]string, n), make([]string, n)
	for i, v := range votes {
		views[i], seqs[i], types[i] = v.ViewID, v.SequenceID, int64(v.MsgType)
		dg[i], ids[i] = v.Digest, v.NodeID
	}
	d, id := packStrings(dg), packStrings(ids)
	sv, sl, sd := stateColumns(states)
	res := VoteResult{Digests: make([][32]byte, n)}
	sbm, mbm := make([]byte, (n+7)/8+1), make([]byte, (n+7)/8+1)
	err := call(func() C.int { return C.pbftv_flush_votes(x.c, C.uint64_t(n), i64(views), i64(seqs), u8(d.blob), u64(d.off), u32(d.ln),
		u8(id.blob), u64(id.off), u32(id.ln), i64(types), sigPtr(sigs), u32(keyIdx), C.uint32_t(len(states)),
		i64(sv), i64(sl), digestPtr(sd), u32(stateIdx), digestPtr(res.Digests), u8(sbm), u8(mbm)) })
	if err != nil {
		return VoteResult{}, err
	}
	res.SigOK, res.MsgOK = bits(sbm, n), bits(mbm, n)
	return res, nil
}

// RequestResult is the outcome of FlushRequests.
type RequestResult struct {
	Digests          [][32]byte // SHA-256 of the request as sent (the client's signed preimage)
	SigOK            []bool
	ConsensusDigests [][32]byte // digest(request with SequenceID = assigned[i]): StartConsensus (pbft_impl.go:67-73)
}

// FlushRequests replaces resolveRequestMsg's per-request StartConsensus
// digests (pbft/network/node.go:521-538) and checks the clients' signatures.
// assigned may be nil (no consensus digests).
func (x *Ctx) FlushRequests(reqs []RequestMsg, sigs [][64]byte, keyIdx []uint32, assigned []int64) (RequestResult,
	error) {
	n := len(reqs)
	if n == 0 {
		return RequestResult{}, nil
	}
	if len(sigs) != n || len(keyIdx) != n || (assigned != nil && len(assigned) != n) {
		return RequestResult{}, &Error{Code: EINVAL, Msg: "column lengths differ"}
	}
	ts, seqs := make([]int64, n), make([]int64, n)
	cids, ops := make([]string, n), make([]string, n)
	for i, r := range reqs {
		ts[i], seqs[i], cids[i], ops[i] = r.Timestamp, r.SequenceID, r.ClientID, r.Operation
	}
	cid, op := packStrings(cids), packStrings(ops)
	res := RequestResult{Digests: make([][32]byte, n)}
	var cons *C.uint8_t
	if assigned != nil {
		res.ConsensusDigests = make([][32]byte, n)
		cons = digestPtr(res.ConsensusDigests)
	}
	sbm := make([]byte, (n+7)/8+1)
	err := call(func() C.int { return C.pbftv_flush_requests(x.c, C.uint64_t(n), i64(ts), u8(cid.blob), u64(cid.off), u32(cid.ln), u8(op.blob),
		u64(op.off), u32(op.ln), i64(seqs), sigPtr(sigs), u32(keyIdx), i64(assigned), digestPtr(res.Digests),
		u8(sbm), cons) })
	if err != nil {
		return RequestResult{}, err
	}
	res.SigOK = bits(sbm, n)
	return res, nil
}

// FlushReplies checks the replicas' signatures on a snapshot of replies (the
// client's reply collection; the reference never checks them, node.go:269-274).
func (x *Ctx) FlushReplies(reps []ReplyMsg, sigs [][64]byte, keyIdx []uint32) ([][32]byte, []bool, error) {
	n := len(reps)
	if n == 0 {
		return nil, nil, nil
	}
	if len(sigs) != n || len(keyIdx) != n {
		return nil, nil, &Error{Code: EINVAL, Msg: "column lengths differ"}
	}
	views, ts := make([]int64, n), make([]int64, n)
	cids, ids, results := make([]string, n), make([]string, n), make([]string, n)
	for i, r := range reps {
		views[i], ts[i], cids[i], ids[i], results[i] = r.ViewID, r.Timestamp, r.ClientID, r.NodeID, r.Result
	}
	cid, id, rs := packStrings(cids), packStrings(ids), packStrings(results)
	dg := make([][32]byte, n)
	sbm := make([]byte, (n+7)/8+1)
	err := call(func() C.int { return C.pbftv_flush_replies(x.c, C.uint64_t(n), i64(views), i64(ts), u8(cid.blob), u64(cid.off), u32(cid.ln),
		u8(id.blob), u64(id.off), u32(id.ln), u8(rs.blob), u64(rs.off), u32(rs.ln), sigPtr(sigs), u32(keyIdx),
		digestPtr(dg), u8(sbm)) })
	if err != nil {
		return nil, nil, err
	}
	return dg, bits(sbm, n), nil
}

// PrePrepareResult is the outcome of FlushPrePrepares.
type PrePrepareResult struct {
	Digests    [][32]byte // SHA-256(json.Marshal(pre-prepare)): the primary's signed preimage
	ReqDigests [][32]byte // digest(embedded request), Hash("null") when it is nil
	SigOK      []bool
	MsgOK      []bool // State.PrePrepare's verifyMsg with ReqMsg = the embedded request
}

// FlushPrePrepares replaces resolvePrePrepareMsg's per-message State.PrePrepare
// (pbft/network/node.go:540-557, pbft_impl.go:91-109).  Only ViewID and
// LastSequenceID of the states are read (the request digest is the embedded
// request's).
func (x *Ctx) FlushPrePrepares(pps []PrePrepareMsg, sigs [][64]byte, keyIdx []uint32, states []State,
	stateIdx []uint32) (PrePrepareResult, error) {
	n := len(pps)
	if n == 0 {
		return PrePrepareResult{}, nil
	}
	if len(sigs) != n || len(keyIdx) != n || len(stateIdx) != n {
		return PrePrepareResult{}, &Error{Code: EINVAL, Msg: "column lengths differ"}
	}
	views, seqs, rts, rseqs := make([]int64, n), make([]int64, n), make([]int64, n), make([]int64, n)
	has := make([]byte, n+1)
	dg, cids, ops := make([]string, n), make([]string, n), make([]string, n)
	for i, p := range pps {
		views[i], seqs[i], dg[i] = p.ViewID, p.SequenceID, p.Digest
		if p.RequestMsg != nil {
			has[i] = 1
			rts[i], rseqs[i] = p.RequestMsg.Timestamp, p.RequestMsg.SequenceID
			cids[i], ops[i] = p.RequestMsg.ClientID, p.RequestMsg.Operation
		}
	}
	d, cid, op := packStrings(dg), packStrings(cids), packStrings(ops)
	sv, sl, _ := stateColumns(states)
	res := PrePrepareResult{Digests: make([][32]byte, n), ReqDigests: make([][32]byte, n)}
	sbm, mbm := make([]byte, (n+7)/8+1), make([]byte, (n+7)/8+1)
	err := call(func() C.int { return C.pbftv_flush_preprepares(x.c, C.uint64_t(n), i64(views), i64(seqs), u8(d.blob), u64(d.off), u32(d.ln),
		u8(has), i64(rts), u8(cid.blob), u64(cid.off), u32(cid.ln), u8(op.blob), u64(op.off), u32(op.ln), i64(rseqs),
		sigPtr(sigs), u32(keyIdx), C.uint32_t(len(states)), i64(sv), i64(sl), u32(stateIdx), digestPtr(res.Digests),
		digestPtr(res.ReqDigests), u8(sbm), u8(mbm)) })
	if err != nil {
		return PrePrepareResult{}, err
	}
	res.SigOK, res.MsgOK = bits(sbm, n), bits(mbm, n)
	return res, nil
}
