// pkg/gpu/gpu.go — cgo binding of libnydusgpu.so (include/nydus_gpu.h) for
// nydus-snapshotter's pkg/converter: the drop-in for the chunk digest + dedup
// stage that `nydus-image create` runs today (pkg/converter/tool/builder.go:148-178,
// pkg/converter/convert_unix.go:443-539).
//
// NOT COMPILED HERE: this container has no Go toolchain (SURVEY.md §8(c)).
// The C ABI it binds is exercised from C (tests/cpp/abi_client.c), C++
// (tests/cpp/converter_test.cpp) and Python ctypes (tests/). Copy this
// directory to pkg/gpu of the reference tree and apply ../converter.patch.
package gpu

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/nydus-gpu/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/nydus-gpu/lib -lnydusgpu -Wl,-rpath,$ORIGIN
#include <stdlib.h>
#include <string.h>
#include "nydus_gpu.h"

// ngpu_read_at_fn over C memory (Unpack reads the nydus stream through it).
typedef struct { const uint8_t *p; uint64_t n; } mem_src;
static int64_t mem_read_at(void *ctx, void *dst, uint64_t n, uint64_t off) {
	const mem_src *s = (const mem_src *)ctx;
	if (off >= s->n) return -1;
	if (n > s->n - off) n = s->n - off;
	memcpy(dst, s->p + off, n);
	return (int64_t)n;
}
static ngpu_read_at_fn mem_reader(void) { return mem_read_at; }
*/
import "C"

import (
	"bytes"
	"context"
	"encoding/hex"
	"errors"
	"fmt"
	"io"
	"os"
	"runtime"
	"strings"
	"sync"
	"sync/atomic"
	"unsafe"

	"github.com/opencontainers/go-digest"
)

type Engine struct{ e *C.ngpu_engine }

// Digest algorithms (PackOption.Digester).
const (
	Blake3 = C.NGPU_DIGEST_BLAKE3
	Sha256 = C.NGPU_DIGEST_SHA256
)

func errOf(e *C.ngpu_engine, rc C.int, what string) error {
	if rc == 0 {
		return nil
	}
	msg := ""
	if e != nil {
		msg = C.GoString(C.ngpu_last_error(e))
	}
	return fmt.Errorf("gpu %s: code %d: %s", what, int(rc), msg)
}

// Engine flags (ngpu_config.flags).
const AlignedChunk = C.NGPU_FLAG_ALIGNED_CHUNK // PackOption.AlignedChunk (builder.go:131-133)

// New mirrors the PackOption fields the stage consumes (pkg/converter/types.go:58-90).
func New(device int, digester, chunkSize, fsVersion, flags uint32) (*Engine, error) {
	cfg := C.ngpu_config{device: C.int32_t(device), digester: C.uint32_t(digester),
		chunk_size: C.uint32_t(chunkSize), fs_version: C.uint32_t(fsVersion), flags: C.uint32_t(flags)}
	var e *C.ngpu_engine
	if rc := C.ngpu_create(&cfg, &e); rc != 0 {
		return nil, errOf(nil, rc, "create")
	}
	return &Engine{e}, nil
}

func (g *Engine) Close() { C.ngpu_destroy(g.e) }

// ChunkDict is `--chunk-dict bootstrap=P` (pkg/converter/tool/builder.go:122-124) as a
// reference-counted HBM object: every Pack opened with it keeps its own reference, and the
// engine caches opens of an unchanged file, so 1000 Packs against one ChunkDictPath load it once.
type ChunkDict struct{ d *C.ngpu_dict }

// OpenChunkDict fails (NGPU_EINVAL) for a bootstrap whose digester, chunk size or RAFS version
// differs from the engine's, as nydus-image rejects it: FsVersion "6" takes RAFS v6 bootstraps,
// FsVersion "5" RAFS v5 ones (every file's chunk infos, in inode-table order).
func (g *Engine) OpenChunkDict(bootstrap string) (*ChunkDict, error) {
	p := C.CString(bootstrap)
	defer C.free(unsafe.Pointer(p))
	var d *C.ngpu_dict
	if rc := C.ngpu_dict_open(g.e, p, &d); rc != 0 {
		return nil, errOf(g.e, rc, "chunk dict")
	}
	return &ChunkDict{d}, nil
}

func (d *ChunkDict) Release() {
	if d != nil {
		C.ngpu_dict_release(d.d)
	}
}

// Pinned returns engine-owned pinned host memory: tar bytes handed to async
// DMA must not live on the Go heap (cgo pointer rules).
func (g *Engine) Pinned(n uint64) ([]byte, error) {
	var p unsafe.Pointer
	if rc := C.ngpu_alloc_pinned(g.e, C.uint64_t(n), &p); rc != 0 {
		return nil, errOf(g.e, rc, "pinned alloc")
	}
	return unsafe.Slice((*byte)(p), n), nil
}

type Chunk = C.ngpu_chunk   // 24 B: offset, length, file_index, file_offset
type Result = C.ngpu_result // 64 B: digest[32], kind, index, ref, blob_index, uncompressed_offset

// PackTar digests and dedups one uncompressed layer tar held in pinned memory.
func (g *Engine) PackTar(tar []byte) ([]Chunk, []Result, error) {
	var pc *C.ngpu_chunk
	var pr *C.ngpu_result
	var n C.uint64_t
	var st C.ngpu_layer_stats
	rc := C.ngpu_pack_tar(g.e, unsafe.Pointer(&tar[0]), C.uint64_t(len(tar)), &pc, &pr, &n, &st)
	if rc != 0 {
		return nil, nil, errOf(g.e, rc, "pack")
	}
	defer C.ngpu_free_host(unsafe.Pointer(pc))
	defer C.ngpu_free_host(unsafe.Pointer(pr))
	chunks := append([]Chunk(nil), unsafe.Slice(pc, int(n))...)
	results := append([]Result(nil), unsafe.Slice(pr, int(n))...)
	return chunks, results, nil
}

// Pack mirrors converter.Pack (convert_unix.go:325): the caller writes the
// uncompressed layer tar, Close() writes the nydus formatted stream
// (`data | tar_header | ... | toc | tar_header`) to dest.  The library writes
// the stream to a file descriptor (ngpu_write_fd); a pipe + goroutine carries
// it to dest, as the FIFO does in packFromTar (convert_unix.go:454-496).
//
// Every way a Pack can end releases it exactly once (packState.end): Close;
// a failed Write / ReadFrom; a source read error inside ReadFrom; ctx.Done()
// -- also when no Write or Close ever comes again, which is what the
// reference's LayerConvertFunc does on its error paths (convert_unix.go:
// 885-907 skips tw.Close() after a copy error or ctx.Done()); and, as a last
// resort, a finalizer when the writer becomes unreachable unclosed (the
// tr.Close() error path, with a context that is never cancelled).  The
// library's retained HBM layer, pinned staging slots and emitter thread and
// this package's pipe goroutine all go with it.
type PackWriter struct {
	s    *packState
	g    *C.ngpu_engine
	Part int // node index of the engine the Pack runs on (-1: a single engine)
}

// packState is what the AfterFunc and the finalizer reach (never the
// PackWriter itself, so that an unclosed writer can become unreachable).
type packState struct {
	mu     sync.Mutex // held across every library call on p
	p      *C.ngpu_pack
	opt    C.ngpu_blob_options
	cancel *C.int32_t // C memory: the library polls it (ngpu_pack_set_cancel)
	stop   func() bool
	refs   int      // holders of cancel: the pack side and the AfterFunc side
	pw     *os.File // the stream's pipe: the library writes, a goroutine copies to dest
	copied chan error
}

// end releases the pack if it is still open (abort: it has not been
// finished), closes the pipe so the copy goroutine ends, and drops the pack
// side's hold on the cancel flag.  Called with mu held.
func (s *packState) end(abort bool) {
	if s.p != nil && abort {
		C.ngpu_pack_abort(s.p)
	}
	s.p = nil
	if s.pw != nil {
		s.pw.Close()
		s.pw = nil
	}
	if s.opt.prefetch_patterns != nil {
		C.free(unsafe.Pointer(s.opt.prefetch_patterns))
		s.opt.prefetch_patterns = nil
	}
	if s.stop != nil {
		if s.stop() { // the AfterFunc will never run: its hold goes too
			s.refs--
		}
		s.stop = nil
		s.unrefFlag()
	}
}

func (s *packState) unrefFlag() { // mu held
	if s.refs--; s.refs == 0 {
		C.free(unsafe.Pointer(s.cancel))
		s.cancel = nil
	}
}

// Pack opens a streaming pack against dict (nil = no chunk dict) on this engine.  ctx.Done() --
// including PackOption.Timeout's deadline, builder.go:153-158 -- stores 1 into the cancel flag
// (the running Write/ReadFrom/Close fails with NGPU_ECANCELED at its next staging slot, as a
// killed builder fails the reference's Pack) and then releases the pack.
// fsVersion 5 or 6 picks the bootstrap format; prefetch is PackOption.PrefetchPatterns (the
// builder's stdin, "" = "/"), written as the bootstrap's prefetch table.
// The output is given at open (ngpu_pack_set_output, ABI 4): the library writes the stream while
// the tar is still arriving, so the layer digest's sequential SHA-256 overlaps the copies and
// digests (DESIGN.md §3 "Early emission").  ociRef = PackOption.OCIRef (NGPU_PACK_OCIREF): Write
// then takes the ORIGINAL gzip layer and dict must be nil (targz-ref, builder.go:180-218).
func (g *Engine) Pack(ctx context.Context, dest io.Writer, compressor, fsVersion uint32, prefetch string,
	dict *ChunkDict, ociRef bool) (*PackWriter, error) {
	var p *C.ngpu_pack
	if rc := C.ngpu_pack_open_dict(g.e, dictOf(dict), packFlags(ociRef), &p); rc != 0 {
		return nil, errOf(g.e, rc, "pack open")
	}
	return startPack(ctx, p, -1, dest, compressor, fsVersion, prefetch)
}

func dictOf(d *ChunkDict) *C.ngpu_dict {
	if d == nil {
		return nil
	}
	return d.d
}

func packFlags(ociRef bool) C.uint32_t {
	if ociRef {
		return C.NGPU_PACK_OCIREF // no chunk data in the stream: nothing to retain
	}
	return C.NGPU_PACK_RETAIN
}

func startPack(ctx context.Context, p *C.ngpu_pack, part int, dest io.Writer, compressor, fsVersion uint32,
	prefetch string) (*PackWriter, error) {
	e := C.ngpu_pack_engine(p)
	s := &packState{p: p, refs: 2, copied: make(chan error, 1),
		cancel: (*C.int32_t)(C.calloc(1, 4)),
		opt: C.ngpu_blob_options{compressor: C.uint32_t(compressor), fs_version: C.uint32_t(fsVersion),
			prefetch_patterns: C.CString(prefetch)}}
	C.ngpu_pack_set_cancel(p, s.cancel)
	s.mu.Lock()
	defer s.mu.Unlock()
	s.stop = context.AfterFunc(ctx, func() {
		atomic.StoreInt32((*int32)(unsafe.Pointer(s.cancel)), 1) // a running call returns soon
		s.mu.Lock()
		defer s.mu.Unlock()
		s.end(true) // (after Close it finds nothing left to release)
		s.unrefFlag()
	})
	r, pw, err := os.Pipe()
	if err != nil {
		s.end(true)
		return nil, err
	}
	s.pw = pw
	copied := s.copied
	go func() { _, err := io.Copy(dest, r); r.Close(); copied <- err }()
	if rc := C.ngpu_pack_set_output(p, &s.opt, C.ngpu_write_fn(C.ngpu_write_fd),
		unsafe.Pointer(uintptr(pw.Fd()))); rc != 0 {
		err := errOf(e, rc, "pack output")
		s.end(true)
		<-copied
		return nil, err
	}
	w := &PackWriter{s: s, g: e, Part: part}
	runtime.SetFinalizer(w, func(w *PackWriter) {
		w.s.mu.Lock()
		w.s.end(true)
		w.s.mu.Unlock()
	})
	return w, nil
}

func (w *PackWriter) ended() error {
	return fmt.Errorf("gpu pack: %w", errPackEnded)
}

var errPackEnded = errors.New("pack ended (cancelled, failed or closed)")

// Write copies synchronously into engine-pinned staging (no Go pointer is retained).
func (w *PackWriter) Write(b []byte) (int, error) {
	s := w.s
	s.mu.Lock()
	defer s.mu.Unlock()
	if s.p == nil {
		return 0, w.ended()
	}
	if len(b) == 0 {
		return 0, nil
	}
	if rc := C.ngpu_pack_write(s.p, unsafe.Pointer(&b[0]), C.uint64_t(len(b))); rc != 0 {
		err := errOf(w.g, rc, "pack write")
		s.end(true) // a failed write leaves the pack open
		return 0, err
	}
	return len(b), nil
}

// ReadFrom lets io.Copy(w, src) -- how packLayer and LayerConvertFunc feed a Pack
// (converter_test.go:283-291, convert_unix.go:870-914) -- read the tar straight into the
// engine's pinned staging (ngpu_pack_reserve / ngpu_pack_commit): the reader fills C memory, so
// there is neither io.Copy's intermediate buffer nor Write's copy into staging.  The source reads
// into the pack's staging, so the pack stays held (mu) while src.Read runs; a ctx.Done() meanwhile
// takes effect when that read returns.  A source error ends the pack: LayerConvertFunc will not
// call Close after it (convert_unix.go:894-897).
func (w *PackWriter) ReadFrom(src io.Reader) (int64, error) {
	s := w.s
	s.mu.Lock()
	defer s.mu.Unlock()
	var total int64
	for {
		if s.p == nil {
			return total, w.ended()
		}
		var p unsafe.Pointer
		var avail C.uint64_t
		if rc := C.ngpu_pack_reserve(s.p, &p, &avail); rc != 0 {
			err := errOf(w.g, rc, "pack reserve")
			s.end(true)
			return total, err
		}
		n, err := src.Read(unsafe.Slice((*byte)(p), int(avail)))
		if n > 0 {
			if rc := C.ngpu_pack_commit(s.p, C.uint64_t(n)); rc != 0 {
				e := errOf(w.g, rc, "pack commit")
				s.end(true)
				return total, e
			}
			total += int64(n)
		}
		if err == io.EOF {
			return total, nil
		}
		if err != nil {
			s.end(true)
			return total, err
		}
	}
}

// Close runs the final dedup, writes the rest of the stream and returns the layer digest
// (sha256 of the stream).
func (w *PackWriter) Close() (digest.Digest, error) {
	s := w.s
	s.mu.Lock()
	defer s.mu.Unlock()
	runtime.SetFinalizer(w, nil)
	if s.p == nil {
		return "", w.ended()
	}
	var pc *C.ngpu_chunk
	var pr *C.ngpu_result
	var n C.uint64_t
	var st C.ngpu_layer_stats
	var info C.ngpu_blob_info
	rc := C.ngpu_pack_finish(s.p, nil, nil, nil, &pc, &pr, &n, &st, &info) // releases it
	copied := s.copied
	s.end(false)
	if err := <-copied; err != nil && rc == 0 {
		return "", err
	}
	if rc != 0 {
		return "", errOf(w.g, rc, "pack close")
	}
	C.ngpu_free_host(unsafe.Pointer(pc))
	C.ngpu_free_host(unsafe.Pointer(pr))
	sum := C.GoBytes(unsafe.Pointer(&info.stream_digest[0]), 32)
	return digest.NewDigestFromEncoded(digest.SHA256, hex.EncodeToString(sum)), nil
}

// RafsBlob is a targz-ref layer's entry of Merge's --blob-digests / --blob-sizes /
// --blob-toc-digests (convert_unix.go:577-590, builder.go:242-253): the hex digest and size of its
// RAFS blob (the nydus stream) and the hex sha256 of its TOC entry data (calcBlobTOCDigest).
type RafsBlob struct {
	Digest    string
	Size      int64
	TOCDigest string
}

// Merge replaces tool.Merge (builder.go:220-294): bootstraps are the layers'
// image.boot entries (read with the reference's own UnpackEntry), names the
// bootstrap file names Merge gives nydus-image (Digest.Hex(), or
// OriginalDigest.Hex() for a targz-ref layer, getBootstrapPath), lowest layer
// first; parentBoot is ParentBootstrapPath's contents (nil = none), prefetch
// MergeOption.PrefetchPatterns; rafs[l] is non-nil for a targz-ref layer (nil
// slice: none).  Returns the merged bootstrap (the overlaid inode tree, RAFS v5
// or v6 as the layers) and the blob ids.
func Merge(boots [][]byte, digests []string, dictBoot, parentBoot []byte, prefetch string,
	rafs []*RafsBlob) ([]byte, []string, error) {
	n := len(boots)
	ptrs := C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0))))
	sizes := C.malloc(C.size_t(n) * 8)
	names := C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0))))
	defer C.free(ptrs)
	defer C.free(sizes)
	defer C.free(names)
	pv := unsafe.Slice((*unsafe.Pointer)(ptrs), n)
	sv := unsafe.Slice((*C.uint64_t)(sizes), n)
	nv := unsafe.Slice((**C.char)(names), n)
	for i := range boots {
		pv[i] = C.CBytes(boots[i])
		defer C.free(pv[i])
		sv[i] = C.uint64_t(len(boots[i]))
		nv[i] = C.CString(digests[i])
		defer C.free(unsafe.Pointer(nv[i]))
	}
	var dict unsafe.Pointer
	if dictBoot != nil {
		dict = C.CBytes(dictBoot)
		defer C.free(dict)
	}
	var mo C.ngpu_merge_options
	if parentBoot != nil {
		mo.parent_bootstrap = C.CBytes(parentBoot)
		mo.parent_size = C.uint64_t(len(parentBoot))
		defer C.free(mo.parent_bootstrap)
	}
	mo.prefetch_patterns = C.CString(prefetch)
	defer C.free(unsafe.Pointer(mo.prefetch_patterns))
	var rd, rs, rt unsafe.Pointer // targz-ref arrays (ngpu_merge_ex2), C memory
	if len(rafs) == n && n > 0 {
		rd = C.calloc(C.size_t(n), C.size_t(unsafe.Sizeof(uintptr(0))))
		rs = C.calloc(C.size_t(n), 8)
		rt = C.calloc(C.size_t(n), C.size_t(unsafe.Sizeof(uintptr(0))))
		defer C.free(rd)
		defer C.free(rs)
		defer C.free(rt)
		rdv := unsafe.Slice((**C.char)(rd), n)
		rsv := unsafe.Slice((*C.uint64_t)(rs), n)
		rtv := unsafe.Slice((**C.char)(rt), n)
		for i, r := range rafs {
			if r == nil {
				continue
			}
			rdv[i] = C.CString(r.Digest)
			defer C.free(unsafe.Pointer(rdv[i]))
			rsv[i] = C.uint64_t(r.Size)
			rtv[i] = C.CString(r.TOCDigest)
			defer C.free(unsafe.Pointer(rtv[i]))
		}
	}
	r, pw, _ := os.Pipe()
	var out bytes.Buffer
	done := make(chan struct{})
	go func() { io.Copy(&out, r); r.Close(); close(done) }()
	var ids *C.char
	rc := C.ngpu_merge_ex2((*unsafe.Pointer)(ptrs), (*C.uint64_t)(sizes), (**C.char)(names),
		C.uint64_t(n), dict, C.uint64_t(len(dictBoot)), &mo, (**C.char)(rd), (*C.uint64_t)(rs),
		(**C.char)(rt), C.ngpu_write_fn(C.ngpu_write_fd), unsafe.Pointer(uintptr(pw.Fd())), &ids)
	pw.Close()
	<-done
	if rc != 0 {
		return nil, nil, fmt.Errorf("gpu merge: code %d: %s", int(rc), C.GoString(C.ngpu_host_error()))
	}
	defer C.ngpu_free_host(unsafe.Pointer(ids))
	return out.Bytes(), strings.Split(C.GoString(ids), ","), nil
}

// Unpack replaces tool.Unpack (`nydus-image unpack`, builder.go:296-362) for
// converter.Unpack (convert_unix.go:669-719): the nydus stream of a layer back
// to its OCI tar, written to dest.  A chunk in a chunk-dict blob fails with
// NGPU_ENOTFOUND (only the layer's own blob is in its stream).
func Unpack(stream []byte, dest io.Writer) error {
	src := (*C.mem_src)(C.malloc(C.size_t(unsafe.Sizeof(C.mem_src{}))))
	defer C.free(unsafe.Pointer(src))
	src.p = (*C.uint8_t)(C.CBytes(stream))
	defer C.free(unsafe.Pointer(src.p))
	src.n = C.uint64_t(len(stream))
	r, pw, err := os.Pipe()
	if err != nil {
		return err
	}
	done := make(chan error, 1)
	go func() { _, err := io.Copy(dest, r); r.Close(); done <- err }()
	rc := C.ngpu_unpack(C.mem_reader(), unsafe.Pointer(src), src.n, C.ngpu_write_fn(C.ngpu_write_fd),
		unsafe.Pointer(uintptr(pw.Fd())))
	pw.Close()
	if err := <-done; err != nil && rc == 0 {
		return err
	}
	if rc != 0 {
		return fmt.Errorf("gpu unpack: code %d: %s", int(rc), C.GoString(C.ngpu_host_error()))
	}
	return nil
}

// DeviceStatus returns the first error a device-pointer stage recorded on the
// GPU since the last check (a digest left unwritten, a bad descriptor), after
// waiting for the engine's streams: *_device calls return before the GPU ends.
func (g *Engine) DeviceStatus() error { return errOf(g.e, C.ngpu_device_status(g.e), "device") }

// Available reports whether the GPU path can be used (NYDUS_GPU=0 disables it).
func Available() bool { return os.Getenv("NYDUS_GPU") != "0" && C.ngpu_device_count() > 0 }

// DeviceCount is the number of gfx950 devices the library sees.
func DeviceCount() int { return int(C.ngpu_device_count()) }

// Node drives every GPU of the host from this process (SURVEY.md §8(e)): one engine per
// device, each Pack on the least-loaded one (north star: the chunk stream is sharded by layer;
// containerd's per-layer goroutines, convert_unix.go:467-538, land on every GPU and every GPU's
// own PCIe link), one chunk dict for all of them -- replicated on every GPU or partitioned by
// digest prefix with the probe exchange over xGMI inside the library.
type Node struct{ n *C.ngpu_node }

func NewNode(devices []int32, digester, chunkSize, fsVersion, flags uint32) (*Node, error) {
	cfg := C.ngpu_config{digester: C.uint32_t(digester), chunk_size: C.uint32_t(chunkSize),
		fs_version: C.uint32_t(fsVersion), flags: C.uint32_t(flags)}
	var n *C.ngpu_node
	if rc := C.ngpu_node_create((*C.int32_t)(unsafe.Pointer(&devices[0])), C.uint32_t(len(devices)), &cfg, &n); rc != 0 {
		return nil, errOf(nil, rc, "node")
	}
	return &Node{n}, nil
}

// OpenChunkDict opens `--chunk-dict bootstrap=P` for every engine of the node.  The library
// caches it per node (an unchanged file opened again returns the same HBM dict), so each Pack can
// open its own reference.  partition=false keeps a full replica on every GPU (no exchange).
func (nd *Node) OpenChunkDict(bootstrap string, partition bool) (*ChunkDict, error) {
	p := C.CString(bootstrap)
	defer C.free(unsafe.Pointer(p))
	mode := C.uint32_t(C.NGPU_NODE_DICT_REPLICATE)
	if partition {
		mode = C.NGPU_NODE_DICT_PARTITION
	}
	var d *C.ngpu_dict
	if rc := C.ngpu_node_dict_open(nd.n, p, mode, &d); rc != 0 {
		return nil, errOf(C.ngpu_node_engine(nd.n, 0), rc, "node chunk dict")
	}
	return &ChunkDict{d}, nil
}

// Engine i of the node.
func (nd *Node) Engine(i int) *Engine { return &Engine{C.ngpu_node_engine(nd.n, C.uint32_t(i))} }

// Pack opens a streaming Pack on the node's least-loaded engine (ngpu_node_pack_open); the
// writer's Part says which.  Arguments and the writer's behaviour are Engine.Pack's.
func (nd *Node) Pack(ctx context.Context, dest io.Writer, compressor, fsVersion uint32, prefetch string,
	dict *ChunkDict, ociRef bool) (*PackWriter, error) {
	var p *C.ngpu_pack
	if rc := C.ngpu_node_pack_open(nd.n, dictOf(dict), packFlags(ociRef), &p); rc != 0 {
		return nil, errOf(C.ngpu_node_engine(nd.n, 0), rc, "node pack open")
	}
	part := -1
	e := C.ngpu_pack_engine(p)
	for i := 0; i < int(C.ngpu_node_size(nd.n)); i++ {
		if C.ngpu_node_engine(nd.n, C.uint32_t(i)) == e {
			part = i
		}
	}
	return startPack(ctx, p, part, dest, compressor, fsVersion, prefetch)
}

// Step runs one node step (ngpu_node_process_step, ABI 5): every device's part
// digested, ONE all-to-all-v of digests to their owners and one of hits back
// (RCCL ncclAllToAllv over xGMI with useRCCL, else peer copies), each part's
// dedup; it returns once everything is enqueued, with no host wait inside.
// parts[i]: device-resident layers on node device i (n = 0: nothing this step).
func (nd *Node) Step(dict *ChunkDict, parts []C.ngpu_node_part, useRCCL bool) error {
	flags := C.uint32_t(0)
	if useRCCL {
		flags = C.NGPU_NODE_STEP_RCCL
	}
	rc := C.ngpu_node_process_step(nd.n, dict.d, &parts[0], C.uint32_t(len(parts)), flags)
	return errOf(C.ngpu_node_engine(nd.n, 0), rc, "node step")
}

func (nd *Node) Close() { C.ngpu_node_destroy(nd.n) }
