// gpuhash.go -- the cgo binding of libmirsha.so (include/mirsha.h) a
// maintainer adds to the reference module, next to processor.go (package
// mirbft, Go 1.14: go.mod:3, .travis.yml:5-6).  It keeps the reference API:
// Processor.Process's signature, Digests[i] for actions.Hash[i]
// (processor.go:129-143), HashResult.Request back-pointers and Go-owned
// 32-byte Digest slices.  Wiring into Processor / ProcessorWorkPool:
// INTEGRATION.md.
//
// There is no Go toolchain in this image or on the GPU boxes, so this file is
// not compiled here.  tests/test_go_binding.py checks on the CPU that every
// C.mirsha_* call and C.MIRSHA_* constant exists in include/mirsha.h with the
// same number of arguments, and that the C mirrors tests/c/cgo_sequence.c and
// tests/c/cgo_path.c (compiled with gcc and run on the GPU) make the same
// calls in the same order.  Go 1.14 idioms only: no unsafe.Slice (Go 1.17);
// C memory is viewed as (*[1 << 40]T)(ptr)[:n:n].
package mirbft

/*
#cgo CFLAGS: -I${SRCDIR}/include
#cgo LDFLAGS: -L${SRCDIR}/lib -lmirsha -Wl,-rpath,${SRCDIR}/lib
#include <stdlib.h>
#include "mirsha.h"
*/
import "C"

import (
	"fmt"
	"hash"
	"runtime"
	"sync"
	"unsafe"
)

// GPUHasher owns one device context, one page-locked arena and one
// page-locked digest buffer (both reused every Ready() cycle, grown on
// demand).  A context is single-caller, so the mutex serialises the batch
// path and the hash.Hash path (ProcessorWorkPool calls its Hasher from
// HashWorkers goroutines, processor.go:312-325).
type GPUHasher struct {
	mu     sync.Mutex
	ctx    *C.mirsha_ctx
	arena  unsafe.Pointer // mirsha_host_alloc: DMA'd at PCIe rate
	cap    int
	dig    unsafe.Pointer // mirsha_host_alloc: the kernel writes the digests here
	digCap int
}

// NewGPUHasher opens device `device` (MIRSHA_ENODEV unless it is a gfx950).
func NewGPUHasher(device int) (*GPUHasher, error) {
	var ctx *C.mirsha_ctx
	if rc := C.mirsha_ctx_create(C.int(device), &ctx); rc != C.MIRSHA_OK {
		return nil, fmt.Errorf("mirsha_ctx_create: %d", int(rc))
	}
	return &GPUHasher{ctx: ctx}, nil
}

// Close releases the pinned buffers and the context.
func (g *GPUHasher) Close() {
	g.mu.Lock()
	defer g.mu.Unlock()
	C.mirsha_host_free(g.arena)
	C.mirsha_host_free(g.dig)
	C.mirsha_ctx_destroy(g.ctx)
	g.arena, g.dig, g.ctx = nil, nil, nil
}

func (g *GPUHasher) fail(rc C.int) {
	// The reference panics on unrecoverable processor failures (processor.go:75,85,91).
	panic(fmt.Sprintf("gpu hashing failed: %d: %s", int(rc), C.GoString(C.mirsha_last_error(g.ctx))))
}

// pinned grows a mirsha_host_alloc buffer to at least n bytes (n >= 1).
func (g *GPUHasher) pinned(p *unsafe.Pointer, cap *int, n int) {
	if n > *cap {
		C.mirsha_host_free(*p)
		*p, *cap = nil, 0
		want := n + n/2
		var q unsafe.Pointer
		if rc := C.mirsha_host_alloc(g.ctx, C.uint64_t(want), &q); rc != C.MIRSHA_OK {
			g.fail(rc)
		}
		*p, *cap = q, want
	}
}

// arenaBytes returns the pinned arena as a Go slice of n bytes (n >= 1).
func (g *GPUHasher) arenaBytes(n int) []byte {
	g.pinned(&g.arena, &g.cap, n)
	return (*[1 << 40]byte)(g.arena)[:n:n]
}

// workers: goroutines for a copy pass.  Capped at 16: the copies are
// memory-bound well before that, and Go 1.14's GOMAXPROCS is the machine's
// CPU count even under a container CPU quota.
func workers(bytes int) int {
	w := runtime.GOMAXPROCS(0)
	if w > 16 {
		w = 16
	}
	if bytes < 1<<20 { // a goroutine start costs more than a small copy
		w = 1
	}
	return w
}

// spread runs fn over [lo, hi) on w goroutines in contiguous parts (wg.Add per part).
func spread(wg *sync.WaitGroup, lo, hi, w int, fn func(a, b int)) {
	if hi <= lo {
		return
	}
	step := (hi - lo + w - 1) / w
	for a := lo; a < hi; a += step {
		b := a + step
		if b > hi {
			b = hi
		}
		wg.Add(1)
		go func(a, b int) {
			defer wg.Done()
			fn(a, b)
		}(a, b)
	}
}

// offsets: off[i], lens[i] of every request (the bytes h.Write sees,
// processor.go:135-137), a two-pass parallel scan; returns the total.
func offsets(reqs []*HashRequest, off []uint64, lens []uint32) int {
	n := len(reqs)
	if n == 0 {
		return 0
	}
	w := workers(n * 64)
	step := (n + w - 1) / w
	sums := make([]uint64, w+1)
	var wg sync.WaitGroup
	spread(&wg, 0, n, w, func(a, b int) {
		s := uint64(0)
		for i := a; i < b; i++ {
			l := 0
			for _, d := range reqs[i].Data {
				l += len(d)
			}
			lens[i] = uint32(l)
			s += uint64(l)
		}
		sums[a/step+1] = s
	})
	wg.Wait()
	for k := 1; k <= w; k++ {
		sums[k] += sums[k-1]
	}
	spread(&wg, 0, n, w, func(a, b int) {
		p := sums[a/step]
		for i := a; i < b; i++ {
			off[i] = p
			p += uint64(lens[i])
		}
	})
	wg.Wait()
	return int(sums[w])
}

// maxBlocks: HashBatch splits a cycle into at most maxBlocks blocks of br
// requests; chunks are runs of whole blocks.
const maxBlocks = 4096

// lengths: lens[i] of every request and each block's starting offset
// bpre[b] (bpre[nb] = the total) in one parallel pass; HashBatch's packing
// goroutines write the offsets themselves, block by block (the second pass of
// offsets() folded into the packing).  No blocks for no requests.
func lengths(reqs []*HashRequest, lens []uint32) (br int, bpre []uint64) {
	n := len(reqs)
	if n == 0 {
		return 1, []uint64{0}
	}
	br = (n + maxBlocks - 1) / maxBlocks
	nb := (n + br - 1) / br
	bpre = make([]uint64, nb+1)
	var wg sync.WaitGroup
	spread(&wg, 0, nb, workers(n*64), func(ba, bb int) {
		for b := ba; b < bb; b++ {
			s := uint64(0)
			for i := b * br; i < n && i < (b+1)*br; i++ {
				l := 0
				for _, d := range reqs[i].Data {
					l += len(d)
				}
				lens[i] = uint32(l)
				s += uint64(l)
			}
			bpre[b+1] = s
		}
	})
	wg.Wait()
	for b := 1; b <= nb; b++ {
		bpre[b] += bpre[b-1]
	}
	return br, bpre
}

// streamPack packs requests [a, b) -- contiguous in the arena from off[a] --
// through a 16 KiB window that streamOut writes with non-temporal stores:
// the copy engine reads lines still dirty in CPU caches ~9% below the link
// rate (profiles/r05o), and plain stores also read every arena line first.
// The C mirror (tests/c/cgo_path.c "nt") measured 7.4 ms per config-2 cycle
// against 9.7 with copy() on the same box (profiles/r05q).
func streamPack(buf []byte, reqs []*HashRequest, off []uint64, a, b int) {
	if a >= b {
		return
	}
	win := make([]byte, 16<<10) // heap: the Go GC does not move it
	at, fill := int(off[a]), 0
	for i := a; i < b; i++ {
		for _, d := range reqs[i].Data {
			if fill+len(d) > len(win) {
				streamOut(buf[at:at+fill], win[:fill])
				at, fill = at+fill, 0
			}
			if len(d) >= len(win) {
				streamOut(buf[at:at+len(d)], d)
				at += len(d)
				continue
			}
			fill += copy(win[fill:], d)
		}
	}
	streamOut(buf[at:at+fill], win[:fill])
}

// streamOut copies src into dst (equal lengths): copy() up to dst's first
// 16-byte boundary and for the last len%64 bytes, ntCopy for the rest.
func streamOut(dst, src []byte) {
	if len(dst) < 128 {
		copy(dst, src)
		return
	}
	h := int(-uintptr(unsafe.Pointer(&dst[0])) & 15)
	copy(dst[:h], src[:h])
	body := (len(dst) - h) &^ 63
	ntCopy(unsafe.Pointer(&dst[h]), unsafe.Pointer(&src[h]), uintptr(body))
	copy(dst[h+body:], src[h+body:])
}

// ntCopy (ntcopy_amd64.s): n bytes, n a multiple of 64, dst 16-byte aligned,
// with MOVNTDQ stores, then SFENCE.
//
//go:noescape
func ntCopy(dst, src unsafe.Pointer, n uintptr)

// chunkEngine: the three calls the chunked HashBatch makes (GPUHasher,
// GPUHasherMulti).
type chunkEngine interface {
	submit(arena unsafe.Pointer, total int, off []uint64, lens []uint32, dig unsafe.Pointer) C.uint64_t
	done(t C.uint64_t) bool
	wait(t C.uint64_t)
}

// chunkBytes: request bytes per full submission.  At BASELINE config 2
// (2^20 x 272 B, 285 MB) a cycle goes in 11 chunks (8 and 16 MiB, then 32):
// the DMA and kernel of chunk k run while chunk k+1 is packed, and the kernel
// writes chunk k's digests straight into the page-locked `dig`
// (tests/c/cgo_path.c, profiles/r05*).
const chunkBytes = 32 << 20

// chunk: requests [lo, hi).  Whole blocks [b0, b1) when b1 > b0; else a part
// of one block larger than a whole budget, its first request at byte `at`.
type chunk struct {
	lo, hi int
	b0, b1 int
	at     uint64
}

// planChunks cuts a cycle into submissions: whole blocks until a quarter, a
// half, then a whole budget is reached (the DMA starts early and the link
// stays busy while the goroutines pack the next, larger chunk).  A block
// holding more than a whole budget (large messages) is cut at request
// boundaries instead, so no submission outgrows one device arena
// (MIRSHA_MAX_DEVICE_ARENA_BYTES: MIRSHA_ERANGE).  tests/c/cgo_path.c and
// tests/test_c_abi.py's plan_chunks are its twins.
func planChunks(n, br int, bpre []uint64, lens []uint32, budgetBytes uint64) []chunk {
	nb := len(bpre) - 1
	req := func(b int) int { // first request of block b
		if b*br > n {
			return n
		}
		return b * br
	}
	var cs []chunk
	for b0 := 0; b0 < nb; {
		budget := budgetBytes
		if k := len(cs); k < 2 {
			budget >>= uint(2 - k)
		}
		if bpre[b0+1]-bpre[b0] > budgetBytes {
			at := bpre[b0]
			for lo, end := req(b0), req(b0+1); lo < end; {
				hi, s := lo+1, uint64(lens[lo])
				for hi < end && s+uint64(lens[hi]) <= budgetBytes {
					s += uint64(lens[hi])
					hi++
				}
				cs = append(cs, chunk{lo: lo, hi: hi, b0: b0, b1: b0, at: at})
				at += s
				lo = hi
			}
			b0++
			continue
		}
		b1 := b0 + 1
		for b1 < nb && bpre[b1]-bpre[b0] < budget && bpre[b1+1]-bpre[b1] <= budgetBytes {
			b1++
		}
		cs = append(cs, chunk{lo: req(b0), hi: req(b1), b0: b0, b1: b1, at: bpre[b0]})
		b0 = b1
	}
	return cs
}

// hashChunked is HashBatch's body: for k = 0..nk the goroutines write the
// offsets of chunk k and pack it (and copy the digests of chunks already back
// into the Go-owned result) while this goroutine submits chunk k-1; then the
// last ticket is waited for and the remaining digests copied.
func hashChunked(e chunkEngine, arena unsafe.Pointer, buf []byte, dig unsafe.Pointer,
	reqs []*HashRequest, off []uint64, lens []uint32, br int, bpre []uint64) []*HashResult {
	n, nb := len(reqs), len(bpre)-1
	total := int(bpre[nb])
	req := func(b int) int {
		if b*br > n {
			return n
		}
		return b * br
	}
	cs := planChunks(n, br, bpre, lens, chunkBytes)
	nk := len(cs)
	digs := (*[1 << 40]byte)(dig)[: 32*n : 32*n]
	digests := make([]byte, 32*n) // Go-owned backing array for every Digest
	tickets := make([]C.uint64_t, nk)
	w := workers(total)
	copied := 0 // chunks whose digests are in `digests`
	for k := 0; k <= nk; k++ {
		var wg sync.WaitGroup
		if k < nk && cs[k].b1 > cs[k].b0 {
			spread(&wg, cs[k].b0, cs[k].b1, w, func(ba, bb int) {
				a, b := req(ba), req(bb)
				p := bpre[ba]
				for i := a; i < b; i++ {
					off[i] = p
					p += uint64(lens[i])
				}
				streamPack(buf, reqs, off, a, b)
			})
		} else if k < nk { // a part of an oversized block: few requests, offsets here
			p := cs[k].at
			for i := cs[k].lo; i < cs[k].hi; i++ {
				off[i] = p
				p += uint64(lens[i])
			}
			spread(&wg, cs[k].lo, cs[k].hi, w, func(a, b int) { streamPack(buf, reqs, off, a, b) })
		}
		upto := copied
		for upto < k-1 && e.done(tickets[upto]) {
			upto++
		}
		if upto > copied {
			spread(&wg, 32*cs[copied].lo, 32*cs[upto].lo, w, func(a, b int) { copy(digests[a:b], digs[a:b]) })
			copied = upto
		}
		if k > 0 {
			lo, hi := cs[k-1].lo, cs[k-1].hi
			tickets[k-1] = e.submit(arena, total, off[lo:hi], lens[lo:hi], unsafe.Pointer(&digs[32*lo]))
		}
		wg.Wait()
	}
	e.wait(tickets[nk-1])
	var wg sync.WaitGroup
	from := n
	if copied < nk {
		from = cs[copied].lo
	}
	spread(&wg, 32*from, 32*n, w, func(a, b int) { copy(digests[a:b], digs[a:b]) })
	wg.Wait()
	results := make([]*HashResult, n)
	for i, r := range reqs {
		results[i] = &HashResult{Request: r, Digest: digests[32*i : 32*i+32 : 32*i+32]}
	}
	return results
}

func (g *GPUHasher) submit(arena unsafe.Pointer, total int, off []uint64, lens []uint32,
	dig unsafe.Pointer) C.uint64_t {
	var t C.uint64_t
	if rc := C.mirsha_submit_batch(g.ctx, (*C.uint8_t)(arena), C.uint64_t(total),
		(*C.uint64_t)(unsafe.Pointer(&off[0])), (*C.uint32_t)(unsafe.Pointer(&lens[0])), C.uint32_t(len(off)),
		(*C.uint8_t)(dig), &t); rc != C.MIRSHA_OK {
		g.fail(rc)
	}
	return t
}

func (g *GPUHasher) done(t C.uint64_t) bool {
	var d C.int
	if rc := C.mirsha_poll(g.ctx, t, &d); rc != C.MIRSHA_OK {
		g.fail(rc)
	}
	return d != 0
}

func (g *GPUHasher) wait(t C.uint64_t) {
	if rc := C.mirsha_wait(g.ctx, t); rc != C.MIRSHA_OK {
		g.fail(rc)
	}
}

// HashBatch returns Digests[i] for reqs[i] (processor.go:133-143 semantics)
// for a whole Ready() cycle, its packing overlapped with the transfer.
func (g *GPUHasher) HashBatch(reqs []*HashRequest) []*HashResult {
	if len(reqs) == 0 {
		return []*HashResult{}
	}
	g.mu.Lock()
	defer g.mu.Unlock()
	off := make([]uint64, len(reqs)) // Go memory without Go pointers: passable to C
	lens := make([]uint32, len(reqs))
	br, bpre := lengths(reqs, lens)
	buf := g.arenaBytes(int(bpre[len(bpre)-1]) + 1)
	g.pinned(&g.dig, &g.digCap, 32*len(reqs))
	return hashChunked(g, g.arena, buf, g.dig, reqs, off, lens, br, bpre)
}

// Hasher returns a Hasher (processor.go:21) for single-message callers:
// Processor.Hasher (processor.go:58) and testengine's Recorder.Hasher
// (testengine/recorder.go:28, 278, 682) take it unchanged.
func (g *GPUHasher) Hasher() Hasher {
	return func() hash.Hash { return &gpuHash{g: g} }
}

// gpuHash is a hash.Hash: Write buffers (multi-slice Write == concatenation),
// Sum runs one SHA-256 on the GPU.  Write never fails, as hash.Hash requires.
type gpuHash struct {
	g   *GPUHasher
	buf []byte
}

func (h *gpuHash) Write(p []byte) (int, error) { h.buf = append(h.buf, p...); return len(p), nil }
func (h *gpuHash) Reset()                      { h.buf = h.buf[:0] }
func (h *gpuHash) Size() int                   { return 32 }
func (h *gpuHash) BlockSize() int              { return 64 }

func (h *gpuHash) Sum(b []byte) []byte {
	h.g.mu.Lock()
	defer h.g.mu.Unlock()
	n := len(h.buf)
	buf := h.g.arenaBytes(n + 1)
	copy(buf, h.buf)
	var off C.uint64_t
	l := C.uint32_t(n)
	var d [32]byte
	if rc := C.mirsha_hash_batch(h.g.ctx, (*C.uint8_t)(h.g.arena), C.uint64_t(n), &off, &l, 1,
		(*C.uint8_t)(unsafe.Pointer(&d[0]))); rc != C.MIRSHA_OK {
		h.g.fail(rc)
	}
	return append(b, d[:]...) // Sum appends and leaves the state unchanged
}

// SubmitBatch packs reqs into the pinned arena and queues their hashing; the
// caller may mutate or drop reqs' Data at once (the library copies the bytes
// into its own staging before returning).  dedup: identical requests
// (epoch-change acks, epoch_target.go:459-477) are hashed once.  The
// ProcessorWorkPool form (processor.go:447-470): submit before the WAL /
// network section, Wait after it.
func (g *GPUHasher) SubmitBatch(reqs []*HashRequest, dedup bool) *PendingBatch {
	n := len(reqs)
	pb := &PendingBatch{reqs: reqs}
	if n == 0 {
		return pb
	}
	g.mu.Lock()
	defer g.mu.Unlock()
	_, off, lens := packAll(g.arenaBytes, reqs)
	ptrs, slen, first, free := sliceArrays(g.arena, off, lens)
	defer free()
	pb.out = C.malloc(C.size_t(32 * n))
	flags := C.int(0)
	if dedup {
		flags = C.MIRSHA_SUBMIT_DEDUP
	}
	if rc := C.mirsha_submit_slices(g.ctx, &ptrs[0], &slen[0], &first[0], C.uint32_t(n),
		(*C.uint8_t)(pb.out), flags, &pb.ticket); rc != C.MIRSHA_OK {
		C.free(pb.out)
		g.fail(rc)
	}
	pb.wait = func() {
		g.mu.Lock()
		rc := C.mirsha_wait(g.ctx, pb.ticket)
		g.mu.Unlock()
		if rc != C.MIRSHA_OK {
			g.fail(rc)
		}
	}
	return pb
}

// packAll copies every request into the arena (grown by grow) at off[i]
// (offsets() first); returns the arena slice, off and lens.
func packAll(grow func(int) []byte, reqs []*HashRequest) ([]byte, []uint64, []uint32) {
	n := len(reqs)
	off := make([]uint64, n)
	lens := make([]uint32, n)
	total := offsets(reqs, off, lens)
	buf := grow(total + 1)
	var wg sync.WaitGroup
	spread(&wg, 0, n, workers(total), func(a, b int) {
		for i := a; i < b; i++ {
			p := int(off[i])
			for _, d := range reqs[i].Data {
				p += copy(buf[p:], d)
			}
		}
	})
	wg.Wait()
	return buf, off, lens
}

// sliceArrays: one slice per request (its packed bytes, processor.go:135-137)
// as C arrays -- C code may not hold Go pointers, and the library reads them
// before mirsha_submit_slices returns -- with the function that frees them.
func sliceArrays(arena unsafe.Pointer, off []uint64, lens []uint32) ([]*C.uint8_t, []C.uint64_t, []C.uint32_t,
	func()) {
	n := len(off)
	cptr := C.malloc(C.size_t(n) * 8)
	clen := C.malloc(C.size_t(n) * 8)
	cfirst := C.malloc(C.size_t(n+1) * 4)
	ptrs := (*[1 << 30]*C.uint8_t)(cptr)[:n:n]
	slen := (*[1 << 30]C.uint64_t)(clen)[:n:n]
	first := (*[1 << 30]C.uint32_t)(cfirst)[: n+1 : n+1]
	for i := range off {
		ptrs[i] = (*C.uint8_t)(unsafe.Pointer(uintptr(arena) + uintptr(off[i])))
		slen[i] = C.uint64_t(lens[i])
		first[i] = C.uint32_t(i)
	}
	first[n] = C.uint32_t(n)
	return ptrs, slen, first, func() {
		C.free(cptr)
		C.free(clen)
		C.free(cfirst)
	}
}

// PendingBatch must be Waited: the library writes pb.out when the ticket
// retires (mirsha_wait, or a fifth submission reusing its ring slot), so the
// C buffer is freed only after Wait.
type PendingBatch struct {
	reqs   []*HashRequest
	out    unsafe.Pointer
	ticket C.uint64_t
	wait   func() // mirsha_wait / mirsha_wait_multi under the hasher's lock
}

// Wait returns Digests[i] for reqs[i], origin order.
func (pb *PendingBatch) Wait() []*HashResult {
	results := make([]*HashResult, len(pb.reqs))
	if len(pb.reqs) == 0 {
		return results
	}
	pb.wait()
	digests := C.GoBytes(pb.out, C.int(32*len(pb.reqs))) // Go-owned copy
	C.free(pb.out)
	for i, r := range pb.reqs {
		results[i] = &HashResult{Request: r, Digest: digests[32*i : 32*i+32 : 32*i+32]}
	}
	return results
}

// GPUHasherMulti: the GPUHasher API over several devices.  Each cycle is
// packed chunk by chunk into a portable page-locked arena
// (mirsha_multi_host_alloc); mirsha_submit_arena_multi cuts each chunk into
// contiguous ranges of equal bytes, one per device, each DMA'd over its own
// link, while the goroutines pack the next chunk.  Digests[i] still belongs
// to reqs[i].
type GPUHasherMulti struct {
	mu     sync.Mutex
	m      *C.mirsha_multi
	arena  unsafe.Pointer // mirsha_multi_host_alloc: pinned for every device
	cap    int
	dig    unsafe.Pointer // mirsha_multi_host_alloc: every device's kernels write their digests here
	digCap int
}

// NewGPUHasherMulti opens one context per listed device.
func NewGPUHasherMulti(devices []int) (*GPUHasherMulti, error) {
	if len(devices) == 0 {
		return nil, fmt.Errorf("no devices")
	}
	cdev := (*C.int)(C.malloc(C.size_t(len(devices)) * C.size_t(unsafe.Sizeof(C.int(0)))))
	defer C.free(unsafe.Pointer(cdev))
	ds := (*[1 << 20]C.int)(unsafe.Pointer(cdev))[:len(devices):len(devices)]
	for i, d := range devices {
		ds[i] = C.int(d)
	}
	var m *C.mirsha_multi
	if rc := C.mirsha_multi_create(cdev, C.int(len(devices)), &m); rc != C.MIRSHA_OK {
		return nil, fmt.Errorf("mirsha_multi_create: %d", int(rc))
	}
	return &GPUHasherMulti{m: m}, nil
}

// Close releases the pinned buffers and every device context.
func (g *GPUHasherMulti) Close() {
	g.mu.Lock()
	defer g.mu.Unlock()
	C.mirsha_host_free(g.arena)
	C.mirsha_host_free(g.dig)
	C.mirsha_multi_destroy(g.m)
	g.arena, g.dig, g.m = nil, nil, nil
}

func (g *GPUHasherMulti) fail(rc C.int) {
	panic(fmt.Sprintf("gpu hashing failed: %d: %s", int(rc), C.GoString(C.mirsha_multi_last_error(g.m))))
}

func (g *GPUHasherMulti) pinned(p *unsafe.Pointer, cap *int, n int) {
	if n > *cap {
		C.mirsha_host_free(*p)
		*p, *cap = nil, 0
		want := n + n/2
		var q unsafe.Pointer
		if rc := C.mirsha_multi_host_alloc(g.m, C.uint64_t(want), &q); rc != C.MIRSHA_OK {
			g.fail(rc)
		}
		*p, *cap = q, want
	}
}

func (g *GPUHasherMulti) arenaBytes(n int) []byte {
	g.pinned(&g.arena, &g.cap, n)
	return (*[1 << 40]byte)(g.arena)[:n:n]
}

func (g *GPUHasherMulti) submit(arena unsafe.Pointer, total int, off []uint64, lens []uint32,
	dig unsafe.Pointer) C.uint64_t {
	var t C.uint64_t
	if rc := C.mirsha_submit_arena_multi(g.m, (*C.uint8_t)(arena), C.uint64_t(total),
		(*C.uint64_t)(unsafe.Pointer(&off[0])), (*C.uint32_t)(unsafe.Pointer(&lens[0])), C.uint32_t(len(off)),
		(*C.uint8_t)(dig), &t); rc != C.MIRSHA_OK {
		g.fail(rc)
	}
	return t
}

func (g *GPUHasherMulti) done(t C.uint64_t) bool {
	var d C.int
	if rc := C.mirsha_poll_multi(g.m, t, &d); rc != C.MIRSHA_OK {
		g.fail(rc)
	}
	return d != 0
}

func (g *GPUHasherMulti) wait(t C.uint64_t) {
	if rc := C.mirsha_wait_multi(g.m, t); rc != C.MIRSHA_OK {
		g.fail(rc)
	}
}

// HashBatch: GPUHasher.HashBatch over every device.
func (g *GPUHasherMulti) HashBatch(reqs []*HashRequest) []*HashResult {
	if len(reqs) == 0 {
		return []*HashResult{}
	}
	g.mu.Lock()
	defer g.mu.Unlock()
	off := make([]uint64, len(reqs))
	lens := make([]uint32, len(reqs))
	br, bpre := lengths(reqs, lens)
	buf := g.arenaBytes(int(bpre[len(bpre)-1]) + 1)
	g.pinned(&g.dig, &g.digCap, 32*len(reqs))
	return hashChunked(g, g.arena, buf, g.dig, reqs, off, lens, br, bpre)
}

// SubmitBatch: GPUHasher.SubmitBatch over every device (each device
// deduplicates its own range with dedup set).
func (g *GPUHasherMulti) SubmitBatch(reqs []*HashRequest, dedup bool) *PendingBatch {
	n := len(reqs)
	pb := &PendingBatch{reqs: reqs}
	if n == 0 {
		return pb
	}
	g.mu.Lock()
	defer g.mu.Unlock()
	_, off, lens := packAll(g.arenaBytes, reqs)
	ptrs, slen, first, free := sliceArrays(g.arena, off, lens)
	defer free()
	pb.out = C.malloc(C.size_t(32 * n))
	flags := C.int(0)
	if dedup {
		flags = C.MIRSHA_SUBMIT_DEDUP
	}
	if rc := C.mirsha_submit_slices_multi(g.m, &ptrs[0], &slen[0], &first[0], C.uint32_t(n),
		(*C.uint8_t)(pb.out), flags, &pb.ticket); rc != C.MIRSHA_OK {
		C.free(pb.out)
		g.fail(rc)
	}
	pb.wait = func() {
		g.mu.Lock()
		rc := C.mirsha_wait_multi(g.m, pb.ticket)
		g.mu.Unlock()
		if rc != C.MIRSHA_OK {
			g.fail(rc)
		}
	}
	return pb
}
