package pbftv_test

// How the reference's node adopts the package (compiled by `go test`, not
// run: no Output comment).  Each example is the body a maintainer puts at
// the named call site of 1556174776/simple_pbft.

import (
	"fmt"

	"github.com/simple-pbft-amd/pbftv"
)

// utils/utils.go:13-17 becomes a one-line wrapper with the same signature.
func ExampleHash() {
	digest := pbftv.Hash([]byte(`{"timestamp":1668519246,"clientID":"client1","operation":"printf","sequenceID":1668519247222762700}`))
	fmt.Println(digest) // a63fc9e8... (tests/golden/digest_kats.json, rebuilt from log/node1.log:3,20)
}

// routeMsgWhenAlarmed's PrePrepared branch (pbft/network/node.go:395-406) and
// resolvePrepareMsg (:559-577): the whole GetAllPreMsg snapshot in one call,
// every vote checked (the reference stops at MSGENOUGH and drops the rest),
// then prepared()'s 2f count (pbft_impl.go:207-217) over the accepted votes.
func ExampleCtx_FlushVotes() {
	x, err := pbftv.Default()
	if err != nil {
		return
	}
	var (
		snapshot []pbftv.VoteMsg // node.MsgBuffer.PrepareMsgs.GetAllPreMsg()
		sigs     [][64]byte      // each vote's r||s (the Signature field, DER -> pbftv.DERToRS)
		keyIdx   []uint32        // node.KeyIndex[vote.NodeID]
		state    pbftv.State     // CurrentState: ViewID, LastSequenceID, SHA-256(json.Marshal(ReqMsg))
	)
	stateIdx := make([]uint32, len(snapshot)) // one state today; sequence-keyed pools pass several
	res, err := x.FlushVotes(snapshot, sigs, keyIdx, []pbftv.State{state}, stateIdx)
	if err != nil {
		return
	}
	const f = 1 // pbft_impl.go:37
	accepted := 0
	for i := range snapshot {
		if res.SigOK[i] && res.MsgOK[i] {
			accepted++ // state.MsgLogs.PrepareMsgs[snapshot[i].NodeID] = &snapshot[i]
		}
	}
	if accepted >= 2*f {
		fmt.Println("prepared: broadcast the commit (node.go:207-226)")
	}
}
