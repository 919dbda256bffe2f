// gpuhash_test.go -- what a maintainer runs with the binding in the reference
// module on an MI355X host (`go test -run GPU`).  Not compiled here (no Go
// toolchain); tests/c/cgo_sequence.c makes the same calls from C on the GPU
// with golden digests, and tests/c/cgo_path.c times HashBatch.
//
// Expected digests come from crypto/sha256, the reference's own Hasher
// (processor.go:21, stress_test.go:388).
package mirbft

import (
	"bytes"
	"crypto/sha256"
	"encoding/binary"
	"math/rand"
	"testing"
)

func testRequests(n int, big map[int]int) []*HashRequest {
	rng := rand.New(rand.NewSource(7))
	reqs := make([]*HashRequest, n)
	for i := range reqs {
		l := rng.Intn(600)
		if b, ok := big[i]; ok {
			l = b
		}
		data := make([]byte, l)
		rng.Read(data)
		c, r := make([]byte, 8), make([]byte, 8)
		binary.LittleEndian.PutUint64(c, uint64(i%4))
		binary.LittleEndian.PutUint64(r, uint64(i/4))
		// state_machine.go:313-317: LE64(ClientId), LE64(ReqNo), Data
		reqs[i] = &HashRequest{Data: [][]byte{c, r, data}}
	}
	return reqs
}

func want(req *HashRequest) []byte {
	h := sha256.New()
	for _, d := range req.Data {
		h.Write(d)
	}
	return h.Sum(nil)
}

func check(t *testing.T, reqs []*HashRequest, got []*HashResult) {
	t.Helper()
	if len(got) != len(reqs) {
		t.Fatalf("%d results for %d requests", len(got), len(reqs))
	}
	for i, r := range got {
		if r.Request != reqs[i] { // origin order, back-pointers kept
			t.Fatalf("result %d is not for request %d", i, i)
		}
		if !bytes.Equal(r.Digest, want(reqs[i])) {
			t.Fatalf("digest %d differs", i)
		}
	}
}

func TestGPUHashBatch(t *testing.T) {
	g, err := NewGPUHasher(0)
	if err != nil {
		t.Skip(err)
	}
	defer g.Close()
	for _, n := range []int{0, 1, 17, 4096, 4097, 100003} {
		reqs := testRequests(n, nil)
		check(t, reqs, g.HashBatch(reqs))
	}
	// blocks larger than a chunk budget are cut at request boundaries
	reqs := testRequests(20000, map[int]int{999: 40 << 20, 1999: 33 << 20})
	check(t, reqs, g.HashBatch(reqs))
}

func TestGPUSubmitBatch(t *testing.T) {
	g, err := NewGPUHasher(0)
	if err != nil {
		t.Skip(err)
	}
	defer g.Close()
	reqs := testRequests(800, nil)
	for i := 400; i < 800; i++ { // epoch-change-like duplicates
		reqs[i] = &HashRequest{Data: reqs[i-400].Data}
	}
	a := g.SubmitBatch(reqs, true)
	b := g.SubmitBatch(reqs[:20], false)
	check(t, reqs[:20], b.Wait())
	check(t, reqs, a.Wait())
}

func TestGPUHasher(t *testing.T) {
	g, err := NewGPUHasher(0)
	if err != nil {
		t.Skip(err)
	}
	defer g.Close()
	h := g.Hasher()()
	if got := h.Sum(nil); !bytes.Equal(got, want(&HashRequest{})) { // testengine/recorder_test.go:83
		t.Fatalf("SHA-256(\"\") = %x", got)
	}
	h.Write([]byte("ab"))
	h.Write([]byte("c"))
	abc := sha256.Sum256([]byte("abc"))
	if got := h.Sum([]byte{1}); !bytes.Equal(got, append([]byte{1}, abc[:]...)) {
		t.Fatalf("Sum(abc) = %x", got)
	}
}

func TestGPUHasherMulti(t *testing.T) {
	g, err := NewGPUHasherMulti([]int{0, 0})
	if err != nil {
		t.Skip(err)
	}
	defer g.Close()
	reqs := testRequests(100003, nil)
	check(t, reqs, g.HashBatch(reqs))
	check(t, reqs[:800], g.SubmitBatch(reqs[:800], false).Wait())
}
