package pbftv

// The reference's CPU path, timed the way SURVEY.md §8(d)(i) asks:
// testing.B with b.RunParallel (GOMAXPROCS = every host core) over
// crypto/ecdsa.Verify and over digest() = sha256(json.Marshal(request))
// (pbft/consensus/pbft_impl.go:235-243), beside the library's batch calls on
// the same inputs.  bench.py reports the OpenSSL stand-in where Go is absent.
//
//	go test -run XXX -bench . -benchtime 5s

import (
	"crypto/ecdsa"
	"crypto/elliptic"
	"crypto/rand"
	"crypto/sha256"
	"encoding/hex"
	"encoding/json"
	"fmt"
	"math/big"
	"sync/atomic"
	"testing"
)

type benchSet struct {
	pubs   []*ecdsa.PublicKey
	raw    [][64]byte
	hashes [][32]byte
	sigs   [][64]byte
	keys   []uint32
}

func makeBenchSet(b *testing.B, nKeys, n int) *benchSet {
	b.Helper()
	s := &benchSet{}
	priv := make([]*ecdsa.PrivateKey, nKeys)
	for i := range priv {
		k, err := ecdsa.GenerateKey(elliptic.P256(), rand.Reader)
		if err != nil {
			b.Fatal(err)
		}
		priv[i] = k
		var r [64]byte
		k.PublicKey.X.FillBytes(r[:32])
		k.PublicKey.Y.FillBytes(r[32:])
		s.pubs, s.raw = append(s.pubs, &k.PublicKey), append(s.raw, r)
	}
	for i := 0; i < n; i++ {
		var h [32]byte
		if _, err := rand.Read(h[:]); err != nil {
			b.Fatal(err)
		}
		k := i % nKeys
		r, ss, err := ecdsa.Sign(rand.Reader, priv[k], h[:])
		if err != nil {
			b.Fatal(err)
		}
		var sig [64]byte
		r.FillBytes(sig[:32])
		ss.FillBytes(sig[32:])
		s.hashes, s.sigs, s.keys = append(s.hashes, h), append(s.sigs, sig), append(s.keys, uint32(k))
	}
	return s
}

// BenchmarkGoECDSAVerifyParallel: verifies/s of crypto/ecdsa.Verify on every core.
func BenchmarkGoECDSAVerifyParallel(b *testing.B) {
	s := makeBenchSet(b, 100, 4096)
	var next uint64
	b.ResetTimer()
	b.RunParallel(func(pb *testing.PB) {
		for pb.Next() {
			i := int(atomic.AddUint64(&next, 1)) % len(s.hashes)
			sig := s.sigs[i]
			if !ecdsa.Verify(s.pubs[s.keys[i]], s.hashes[i][:], new(big.Int).SetBytes(sig[:32]),
				new(big.Int).SetBytes(sig[32:])) {
				b.Error("valid signature rejected")
			}
		}
	})
}

// BenchmarkLibraryVerify: the same signatures in batches of 65,536 through
// pbftv_ecdsa_p256_verify_batch (host buffers, PCIe included).
func BenchmarkLibraryVerify(b *testing.B) {
	x, err := Open(0)
	if IsNoDevice(err) {
		b.Skip("no gfx950 GPU")
	}
	if err != nil {
		b.Fatal(err)
	}
	defer x.Close()
	s := makeBenchSet(b, 100, 4096)
	const batch = 65536
	h, sg, k := make([][32]byte, batch), make([][64]byte, batch), make([]uint32, batch)
	for i := 0; i < batch; i++ {
		j := i % len(s.hashes)
		h[i], sg[i], k[i] = s.hashes[j], s.sigs[j], s.keys[j]
	}
	if _, err := x.RegisterKeys(s.raw); err != nil {
		b.Fatal(err)
	}
	b.ResetTimer()
	for done := 0; done < b.N; done += batch {
		ok, err := x.VerifySigs(h, sg, k)
		if err != nil || !ok[0] {
			b.Fatal("library verify failed", err)
		}
	}
}

// BenchmarkGoDigestParallel: digest(request) as the reference computes it,
// json.Marshal + sha256 + hex (utils.Hash), on every core.
func BenchmarkGoDigestParallel(b *testing.B) {
	reqs := make([]*RequestMsg, 1024)
	for i := range reqs {
		reqs[i] = &RequestMsg{Timestamp: int64(1668519246 + i), ClientID: fmt.Sprintf("client%d", i),
			Operation: "printf", SequenceID: int64(1668519247222762700 + i)}
	}
	var next uint64
	b.ResetTimer()
	b.RunParallel(func(pb *testing.PB) {
		for pb.Next() {
			i := int(atomic.AddUint64(&next, 1)) % len(reqs)
			pre, err := json.Marshal(reqs[i])
			if err != nil {
				b.Error(err)
			}
			h := sha256.Sum256(pre)
			_ = hex.EncodeToString(h[:])
		}
	})
}
