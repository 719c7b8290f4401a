// Package pbftv is the cgo binding of libpbftv.so (include/pbftv.h): the
// MI355X batch verifier for the crypto hot path of 1556174776/simple_pbft.
//
// It keeps the reference's call-site signatures where they exist --
// Hash(content []byte) string is utils.Hash (utils/utils.go:13-17) -- and adds
// the batch entry points a pool flush calls with a whole GetAll* snapshot
// (pbft/network/node.go:365-439, 559-598) instead of one verifyMsg per vote.
//
// Every buffer handed to C is caller-owned Go memory without Go pointers
// inside ([N]byte arrays, []int64, []uint32, one packed []byte per string
// column), and the library keeps no pointer after a call returns, so the cgo
// pointer rules hold.  Cryptographic rejection is a false, never an error.
//
// Build: make -C ../../simple_pbft_amd (hipcc, gfx950) first; this package
// links ../../simple_pbft_amd/libpbftv.so.
package pbftv

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../simple_pbft_amd -lpbftv -Wl,-rpath,${SRCDIR}/../../simple_pbft_amd
#include <stdlib.h>
#include "pbftv.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"sync"
	"unsafe"
)

// Error codes of include/pbftv.h.
const (
	EINVAL  = -1
	ENODEV  = -2
	EDEVICE = -3
	ENOMEM  = -4
	ENOKEYS = -5
)

// Error is a nonzero PBFTV_E* return code with the library's message.
type Error struct {
	Code int
	Msg  string
}

func (e *Error) Error() string { return fmt.Sprintf("pbftv error %d: %s", e.Code, e.Msg) }

// call runs one library call and reads its error message on the same OS
// thread: pbftv_last_error is thread-local, and a goroutine can move to
// another thread between two cgo calls.
func call(f func() C.int) error {
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	return check(f())
}

func check(rc C.int) error {
	if rc == 0 {
		return nil
	}
	msg := C.GoString(C.pbftv_last_error())
	if msg == "" {
		msg = C.GoString(C.pbftv_strerror(rc))
	}
	return &Error{Code: int(rc), Msg: msg}
}

// IsNoDevice reports whether err is PBFTV_ENODEV (no usable gfx950 GPU).
func IsNoDevice(err error) bool {
	var e *Error
	return errors.As(err, &e) && e.Code == ENODEV
}

// Ctx is one pbftv_ctx: the GPUs of a device mask.  Safe for concurrent use
// (the library serialises per device).
type Ctx struct {
	c *C.pbftv_ctx
}

// Open opens the GPUs in deviceMask (0 = every visible gfx950 GPU).
func Open(deviceMask uint32) (*Ctx, error) {
	var c *C.pbftv_ctx
	if err := call(func() C.int { return C.pbftv_open(&c, C.uint32_t(deviceMask)) }); err != nil {
		return nil, err
	}
	return &Ctx{c: c}, nil
}

// Close releases the context (its tables and buffers).
func (x *Ctx) Close() {
	if x.c != nil {
		C.pbftv_close(x.c)
		x.c = nil
	}
}

// Devices is the number of GPUs in the context.
func (x *Ctx) Devices() int { return int(C.pbftv_device_count(x.c)) }

var (
	defaultOnce sync.Once
	defaultCtx  *Ctx
	defaultErr  error
)

// Default is the process-wide context on every visible GPU, opened on first use.
// MustInit opens the default context or panics with the library's reason
// (ENODEV: no usable gfx950 GPU).  Call it once at replica start-up.
func MustInit() *Ctx {
	x, err := Default()
	if err != nil {
		panic(fmt.Sprintf("pbftv: the GPU verify path is unavailable (%v); this build has no CPU fallback", err))
	}
	return x
}

func Default() (*Ctx, error) {
	defaultOnce.Do(func() { defaultCtx, defaultErr = Open(0) })
	return defaultCtx, defaultErr
}

func u8(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

func i64(v []int64) *C.int64_t {
	if len(v) == 0 {
		return nil
	}
	return (*C.int64_t)(unsafe.Pointer(&v[0]))
}

func u32(v []uint32) *C.uint32_t {
	if len(v) == 0 {
		return nil
	}
	return (*C.uint32_t)(unsafe.Pointer(&v[0]))
}

func u64(v []uint64) *C.uint64_t {
	if len(v) == 0 {
		return nil
	}
	return (*C.uint64_t)(unsafe.Pointer(&v[0]))
}

func bits(bm []byte, n int) []bool {
	out := make([]bool, n)
	for i := range out {
		out[i] = bm[i/8]>>(uint(i)%8)&1 == 1
	}
	return out
}

// ---------------------------------------------------------------- SHA-256

// Hash keeps utils.Hash's signature (utils/utils.go:13-17): lowercase hex
// SHA-256 of content, on the default context.  utils.Hash cannot fail, so a
// library error panics -- including PBFTV_ENODEV on a host without a gfx950
// GPU: there is deliberately no CPU fallback behind this path.  A replica
// built with the drop-in calls MustInit at start-up, so a GPU-less host fails
// there, before it joins consensus, not in its first digest().
func Hash(content []byte) string {
	x, err := Default()
	if err != nil {
		panic(err)
	}
	s, err := x.Hash(content)
	if err != nil {
		panic(err)
	}
	return s
}

// Hash is utils.Hash on this context.
func (x *Ctx) Hash(content []byte) (string, error) {
	var out [65]C.char
	if err := call(func() C.int { return C.pbftv_hash_hex(x.c, u8(content), C.uint64_t(len(content)), &out[0]) }); err != nil {
		return "", err
	}
	return C.GoString(&out[0]), nil
}

// column packs byte strings as (blob, offsets, lengths): one allocation with
// no Go pointers inside; blob is never empty, so &blob[0] is always valid.
type column struct {
	blob []byte
	off  []uint64
	ln   []uint32
}

func packBytes(items [][]byte) column {
	c := column{off: make([]uint64, len(items)+1), ln: make([]uint32, len(items)+1)}
	for i, s := range items {
		c.off[i], c.ln[i] = uint64(len(c.blob)), uint32(len(s))
		c.blob = append(c.blob, s...)
	}
	c.blob = append(c.blob, 0)
	return c
}

func packStrings(items []string) column {
	c := column{off: make([]uint64, len(items)+1), ln: make([]uint32, len(items)+1)}
	for i, s := range items {
		c.off[i], c.ln[i] = uint64(len(c.blob)), uint32(len(s))
		c.blob = append(c.blob, s...)
	}
	c.blob = append(c.blob, 0)
	return c
}

// HashBatch hashes a whole snapshot in one GPU launch: out[i] = SHA-256(msgs[i]).
func (x *Ctx) HashBatch(msgs [][]byte) ([][32]byte, error) {
	n := len(msgs)
	if n == 0 {
		return nil, nil
	}
	c := packBytes(msgs)
	out := make([][32]byte, n)
	err := call(func() C.int { return C.pbftv_sha256_batch(x.c, u8(c.blob), u64(c.off), u32(c.ln), C.uint64_t(n),
		(*C.uint8_t)(unsafe.Pointer(&out[0]))) })
	return out, err
}

// ---------------------------------------------------------------- keys

func keyPtr(pubXY [][64]byte) *C.uint8_t {
	if len(pubXY) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&pubXY[0]))
}

// RegisterKeys registers the replica public keys (X||Y big-endian: the
// uncompressed elliptic.Marshal encoding without its 0x04 byte) in NodeTable
// order (pbft/network/node.go:60-65); valid[j] = key j is a P-256 point.
func (x *Ctx) RegisterKeys(pubXY [][64]byte) ([]bool, error) {
	valid := make([]byte, len(pubXY)+1)
	if err := call(func() C.int { return C.pbftv_register_keys(x.c, keyPtr(pubXY), C.uint32_t(len(pubXY)), u8(valid)) }); err != nil {
		return nil, err
	}
	out := make([]bool, len(pubXY))
	for i := range out {
		out[i] = valid[i] == 1
	}
	return out, nil
}

// AddKeys appends keys after the registered ones (membership change).
func (x *Ctx) AddKeys(pubXY [][64]byte) ([]bool, error) {
	valid := make([]byte, len(pubXY)+1)
	if err := call(func() C.int { return C.pbftv_add_keys(x.c, keyPtr(pubXY), C.uint32_t(len(pubXY)), u8(valid)) }); err != nil {
		return nil, err
	}
	out := make([]bool, len(pubXY))
	for i := range out {
		out[i] = valid[i] == 1
	}
	return out, nil
}

// SetKey replaces key index in place.
func (x *Ctx) SetKey(index uint32, pubXY [64]byte) (bool, error) {
	var valid C.uint8_t
	err := call(func() C.int { return C.pbftv_set_key(x.c, C.uint32_t(index), (*C.uint8_t)(unsafe.Pointer(&pubXY[0])), &valid) })
	return valid == 1, err
}

// ---------------------------------------------------------------- signatures

// VerifySigs: crypto/ecdsa.Verify(key[keyIdx[i]], hashes[i], r_i, s_i) for
// every i, sigs[i] = r||s big-endian.
func (x *Ctx) VerifySigs(hashes [][32]byte, sigs [][64]byte, keyIdx []uint32) ([]bool, error) {
	n := len(hashes)
	if len(sigs) != n || len(keyIdx) != n {
		return nil, &Error{Code: EINVAL, Msg: "hashes, sigs and keyIdx differ in length"}
	}
	if n == 0 {
		return nil, nil
	}
	bm := make([]byte, (n+7)/8)
	err := call(func() C.int { return C.pbftv_ecdsa_p256_verify_batch(x.c, (*C.uint8_t)(unsafe.Pointer(&hashes[0])),
		(*C.uint8_t)(unsafe.Pointer(&sigs[0])), u32(keyIdx), C.uint64_t(n), u8(bm)) })
	if err != nil {
		return nil, err
	}
	return bits(bm, n), nil
}

// QCVerify verifies one quorum certificate and counts it: reached =
// accepted >= quorum (quorum = 2f reproduces prepared()/committed(),
// pbft/consensus/pbft_impl.go:207-232; 2f+1 checks a PBFT certificate).
func (x *Ctx) QCVerify(hashes [][32]byte, sigs [][64]byte, keyIdx []uint32, quorum uint32) (ok []bool, accepted int,
	reached bool, err error) {
	n := len(hashes)
	if len(sigs) != n || len(keyIdx) != n {
		return nil, 0, false, &Error{Code: EINVAL, Msg: "hashes, sigs and keyIdx differ in length"}
	}
	if n == 0 {
		return nil, 0, quorum == 0, nil
	}
	bm := make([]byte, (n+7)/8)
	var acc C.uint64_t
	var q C.int
	err := call(func() C.int { return C.pbftv_qc_verify(x.c, (*C.uint8_t)(unsafe.Pointer(&hashes[0])), (*C.uint8_t)(unsafe.Pointer(&sigs[0])),
		u32(keyIdx), C.uint64_t(n), C.uint32_t(quorum), u8(bm), &acc, &q) })
	if err != nil {
		return nil, 0, false, err
	}
	return bits(bm, n), int(acc), q != 0, nil
}

// SetLatencyPathMax: batches of up to n signatures take the latency path (one
// wave per signature; up to 128 of them served by the resident armed kernel
// with no launch on the call's path); larger ones the throughput path.  The
// default is 2048; 0 sends every batch to the throughput path.
func (x *Ctx) SetLatencyPathMax(n uint64) error {
	return call(func() C.int { return C.pbftv_set_latency_path_max(x.c, C.uint64_t(n)) })
}

// QCStamps says where the last latency-path call's time went
// (pbftv_qc_stamps): host ns from entry to hand-over (doorbell rung or kernel
// launched) and to return, and whether the armed kernel served it.
type QCStamps struct {
	HandoverNs, TotalNs uint64
	Armed               bool
}

func (x *Ctx) QCStamps() (QCStamps, error) {
	var out [8]C.uint64_t
	err := call(func() C.int { return C.pbftv_qc_stamps(x.c, 0, &out[0]) })
	if err != nil {
		return QCStamps{}, err
	}
	return QCStamps{HandoverNs: uint64(out[0]), TotalNs: uint64(out[1]), Armed: uint64(out[2])&1 == 1}, nil
}

// QCCounters are the latency path's counters on device 0 since Open
// (pbftv_qc_counters): calls, calls an armed kernel served, armed calls rerun
// by a launch (an exceptional signature), signatures through a launched
// kernel's exact path, launches, armings, keeper rotations, and the armed
// kernel now (workgroups, 0 = none; Wide).
type QCCounters struct {
	Calls, Armed, Reruns, ExactSigs, Launches, Armings, Rotations uint64
	ArmedWorkgroups                                              uint32
	Wide                                                         bool
}

func (x *Ctx) QCCounters() (QCCounters, error) {
	var out [8]C.uint64_t
	err := call(func() C.int { return C.pbftv_qc_counters(x.c, 0, &out[0]) })
	if err != nil {
		return QCCounters{}, err
	}
	return QCCounters{Calls: uint64(out[0]), Armed: uint64(out[1]), Reruns: uint64(out[2]), ExactSigs: uint64(out[3]),
		Launches: uint64(out[4]), Armings: uint64(out[5]), Rotations: uint64(out[6]),
		ArmedWorkgroups: uint32(uint64(out[7])), Wide: uint64(out[7])>>32 == 1}, nil
}

// DERToRS is the parse half of crypto/ecdsa.VerifyASN1 (go1.19 cryptobyte
// strictness).  A rejected encoding returns ok = false and r = s = 0, which
// VerifySigs turns into a false, so VerifyASN1(pub, h, der) ==
// VerifySigs(h, DERToRS(der), key).
func DERToRS(der []byte) (rs [64]byte, ok bool) {
	r := C.pbftv_ecdsa_der_to_rs(u8(der), C.uint64_t(len(der)), (*C.uint8_t)(unsafe.Pointer(&rs[0])))
	return rs, r == 1
}

// ---------------------------------------------------------------- Go-JSON preimages (host only)

func cstr(s string) (*C.char, C.uint64_t) {
	if len(s) == 0 {
		return nil, 0
	}
	b := []byte(s)
	return (*C.char)(unsafe.Pointer(&b[0])), C.uint64_t(len(b))
}

func encode(fn func(out *C.uint8_t, capacity C.uint64_t) C.uint64_t) []byte {
	n := fn(nil, 0)
	out := make([]byte, int(n)+1)
	fn(u8(out), n)
	return out[:n]
}

// GoJSONRequest is json.Marshal(&RequestMsg{...}) as the library encodes it.
func GoJSONRequest(m RequestMsg) []byte {
	cid, cidn := cstr(m.ClientID)
	op, opn := cstr(m.Operation)
	return encode(func(out *C.uint8_t, capacity C.uint64_t) C.uint64_t {
		return C.pbftv_gojson_request(C.int64_t(m.Timestamp), cid, cidn, op, opn, C.int64_t(m.SequenceID), out, capacity)
	})
}

// GoJSONVote is json.Marshal(&VoteMsg{...}) as the library encodes it.
func GoJSONVote(m VoteMsg) []byte {
	d, dn := cstr(m.Digest)
	id, idn := cstr(m.NodeID)
	return encode(func(out *C.uint8_t, capacity C.uint64_t) C.uint64_t {
		return C.pbftv_gojson_vote(C.int64_t(m.ViewID), C.int64_t(m.SequenceID), d, dn, id, idn, C.int64_t(m.MsgType),
			out, capacity)
	})
}

// GoJSONReply is json.Marshal(&ReplyMsg{...}) as the library encodes it.
func GoJSONReply(m ReplyMsg) []byte {
	cid, cidn := cstr(m.ClientID)
	id, idn := cstr(m.NodeID)
	res, resn := cstr(m.Result)
	return encode(func(out *C.uint8_t, capacity C.uint64_t) C.uint64_t {
		return C.pbftv_gojson_reply(C.int64_t(m.ViewID), C.int64_t(m.Timestamp), cid, cidn, id, idn, res, resn, out, capacity)
	})
}

// GoJSONPrePrepare is json.Marshal(&PrePrepareMsg{...}) as the library
// encodes it (a nil RequestMsg encodes as null).
func GoJSONPrePrepare(m PrePrepareMsg) []byte {
	d, dn := cstr(m.Digest)
	has, ts, sq := C.int(0), C.int64_t(0), C.int64_t(0)
	var cid, op *C.char
	var cidn, opn C.uint64_t
	if m.RequestMsg != nil {
		has, ts, sq = 1, C.int64_t(m.RequestMsg.Timestamp), C.int64_t(m.RequestMsg.SequenceID)
		cid, cidn = cstr(m.RequestMsg.ClientID)
		op, opn = cstr(m.RequestMsg.Operation)
	}
	return encode(func(out *C.uint8_t, capacity C.uint64_t) C.uint64_t {
		return C.pbftv_gojson_preprepare(C.int64_t(m.ViewID), C.int64_t(m.SequenceID), d, dn, has, ts, cid, cidn, op,
			opn, sq, out, capacity)
	})
}

// VerifyMsgBatch is State.verifyMsg (pbft/consensus/pbft_impl.go:176-202)
// over a snapshot against one state: the request hashed once (st.ReqDigest),
// each digest string compared exactly as Go compares strings.
func VerifyMsgBatch(st State, viewIDs, seqIDs []int64, digestGot []string) ([]bool, error) {
	n := len(digestGot)
	if len(viewIDs) != n || len(seqIDs) != n {
		return nil, &Error{Code: EINVAL, Msg: "column lengths differ"}
	}
	if n == 0 {
		return nil, nil
	}
	c := packStrings(digestGot)
	bm := make([]byte, (n+7)/8+1)
	err := call(func() C.int { return C.pbftv_verify_msg_batch(C.int64_t(st.ViewID), C.int64_t(st.LastSequenceID),
		(*C.uint8_t)(unsafe.Pointer(&st.ReqDigest[0])), C.uint64_t(n), i64(viewIDs), i64(seqIDs),
		(*C.char)(unsafe.Pointer(&c.blob[0])), u64(c.off), u32(c.ln), u8(bm)) })
	if err != nil {
		return nil, err
	}
	return bits(bm, n), nil
}
