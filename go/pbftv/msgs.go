package pbftv

// The reference's message structs, field for field and tag for tag
// (pbft/consensus/pbft_msg_types.go:3-38 of 1556174776/simple_pbft), so that
// encoding/json.Marshal of these values is the digest / signing preimage the
// library rebuilds on the GPU (pbftv_gojson_*, pbftv_flush_*).  A node that
// imports this package passes its own consensus values field by field; these
// copies exist so the package and its tests build without the reference
// module (whose consensus package imports zap).

// RequestMsg mirrors pbft_msg_types.go:3-8.
type RequestMsg struct {
	Timestamp  int64  `json:"timestamp"`
	ClientID   string `json:"clientID"`
	Operation  string `json:"operation"`
	SequenceID int64  `json:"sequenceID"`
}

// ReplyMsg mirrors pbft_msg_types.go:10-16.
type ReplyMsg struct {
	ViewID    int64  `json:"viewID"`
	Timestamp int64  `json:"timestamp"`
	ClientID  string `json:"clientID"`
	NodeID    string `json:"nodeID"`
	Result    string `json:"result"`
}

// PrePrepareMsg mirrors pbft_msg_types.go:18-23.
type PrePrepareMsg struct {
	ViewID     int64       `json:"viewID"`
	SequenceID int64       `json:"sequenceID"`
	Digest     string      `json:"digest"`
	RequestMsg *RequestMsg `json:"requestMsg"`
}

// VoteMsg mirrors pbft_msg_types.go:25-31 (embedded MsgType, tag "msgType").
type VoteMsg struct {
	ViewID     int64  `json:"viewID"`
	SequenceID int64  `json:"sequenceID"`
	Digest     string `json:"digest"`
	NodeID     string `json:"nodeID"`
	MsgType    `json:"msgType"`
}

// MsgType mirrors pbft_msg_types.go:33-38.
type MsgType int

const (
	PrepareMsg MsgType = iota
	CommitMsg
)

// State is what State.verifyMsg (pbft/consensus/pbft_impl.go:176-202) reads
// of a consensus state: its view, the last committed sequence ID (-1 = none)
// and the SHA-256 of Go-JSON(state.MsgLogs.ReqMsg).
type State struct {
	ViewID         int64
	LastSequenceID int64
	ReqDigest      [32]byte
}
