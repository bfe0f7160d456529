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
	"fmt"
	"io"
	"os"
	"strings"
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
type PackWriter struct {
	g      *Engine
	p      *C.ngpu_pack
	dest   io.Writer
	opt    C.ngpu_blob_options
	cancel *C.int32_t // C memory: the library polls it (ngpu_pack_set_cancel)
	stop   func() bool
	pw     *os.File   // the stream's pipe: the library writes, a goroutine copies to dest
	copied chan error
}

// Pack opens a streaming pack against dict (nil = no chunk dict).  ctx.Done() -- including
// PackOption.Timeout's deadline, builder.go:153-158 -- stores 1 into the cancel flag; the running
// Write/Close then fails with NGPU_ECANCELED, as a killed builder fails the reference's Pack.
// fsVersion 5 or 6 picks the bootstrap format; prefetch is PackOption.PrefetchPatterns (the
// builder's stdin, "" = "/"), written as the bootstrap's prefetch table.
// The output is given at open (ngpu_pack_set_output, ABI 4): the library writes the stream while
// the tar is still arriving, so the layer digest's sequential SHA-256 overlaps the copies and
// digests (DESIGN.md §3 "Early emission").  ociRef = PackOption.OCIRef (NGPU_PACK_OCIREF): Write
// then takes the ORIGINAL gzip layer and dict must be nil (targz-ref, builder.go:180-218).
func (g *Engine) Pack(ctx context.Context, dest io.Writer, compressor, fsVersion uint32, prefetch string,
	dict *ChunkDict, ociRef bool) (*PackWriter, error) {
	var p *C.ngpu_pack
	var d *C.ngpu_dict
	if dict != nil {
		d = dict.d
	}
	flags := C.uint32_t(C.NGPU_PACK_RETAIN)
	if ociRef {
		flags = C.NGPU_PACK_OCIREF // no chunk data in the stream: nothing to retain
	}
	if rc := C.ngpu_pack_open_dict(g.e, d, flags, &p); rc != 0 {
		return nil, errOf(g.e, rc, "pack open")
	}
	flag := (*C.int32_t)(C.calloc(1, 4))
	C.ngpu_pack_set_cancel(p, flag)
	stop := context.AfterFunc(ctx, func() { atomic.StoreInt32((*int32)(unsafe.Pointer(flag)), 1) })
	w := &PackWriter{g: g, p: p, dest: dest, cancel: flag, stop: stop, copied: make(chan error, 1),
		opt: C.ngpu_blob_options{compressor: C.uint32_t(compressor), fs_version: C.uint32_t(fsVersion),
			prefetch_patterns: C.CString(prefetch)}} // freed in done()
	r, pw, err := os.Pipe()
	if err != nil {
		C.ngpu_pack_abort(p)
		w.done()
		return nil, err
	}
	w.pw = pw
	go func() { _, err := io.Copy(dest, r); r.Close(); w.copied <- err }()
	if rc := C.ngpu_pack_set_output(p, &w.opt, C.ngpu_write_fn(C.ngpu_write_fd),
		unsafe.Pointer(uintptr(pw.Fd()))); rc != 0 {
		err := errOf(g.e, rc, "pack output")
		C.ngpu_pack_abort(p)
		pw.Close()
		<-w.copied
		w.done()
		return nil, err
	}
	return w, nil
}

func (w *PackWriter) done() {
	C.free(unsafe.Pointer(w.opt.prefetch_patterns))
	w.opt.prefetch_patterns = nil
	if w.stop() { // AfterFunc did not run: nobody touches the flag any more
		C.free(unsafe.Pointer(w.cancel))
	} // else it ran; the flag leaks its 4 bytes rather than racing the store
}

// Write copies synchronously into engine-pinned staging (no Go pointer is retained).
func (w *PackWriter) Write(b []byte) (int, error) {
	if len(b) == 0 {
		return 0, nil
	}
	if rc := C.ngpu_pack_write(w.p, unsafe.Pointer(&b[0]), C.uint64_t(len(b))); rc != 0 {
		err := errOf(w.g.e, rc, "pack write")
		C.ngpu_pack_abort(w.p) // a failed write leaves the pack open
		w.p = nil
		w.done()
		return 0, err
	}
	return len(b), nil
}

// ReadFrom lets io.Copy(w, src) -- how packLayer and LayerConvertFunc feed a Pack
// (converter_test.go:283-291, convert_unix.go:870-914) -- read the tar straight into the
// engine's pinned staging (ngpu_pack_reserve / ngpu_pack_commit): the reader fills C memory, so
// there is neither io.Copy's intermediate buffer nor Write's copy into staging.
func (w *PackWriter) ReadFrom(src io.Reader) (int64, error) {
	var total int64
	for {
		var p unsafe.Pointer
		var avail C.uint64_t
		if rc := C.ngpu_pack_reserve(w.p, &p, &avail); rc != 0 {
			err := errOf(w.g.e, rc, "pack reserve")
			C.ngpu_pack_abort(w.p)
			w.p = nil
			w.done()
			return total, err
		}
		n, err := src.Read(unsafe.Slice((*byte)(p), int(avail)))
		if n > 0 {
			if rc := C.ngpu_pack_commit(w.p, C.uint64_t(n)); rc != 0 {
				e := errOf(w.g.e, rc, "pack commit")
				C.ngpu_pack_abort(w.p)
				w.p = nil
				w.done()
				return total, e
			}
			total += int64(n)
		}
		if err == io.EOF {
			return total, nil
		}
		if err != nil {
			return total, err
		}
	}
}

// Close runs the final dedup, writes the rest of the stream and returns the layer digest
// (sha256 of the stream).
func (w *PackWriter) Close() (digest.Digest, error) {
	var pc *C.ngpu_chunk
	var pr *C.ngpu_result
	var n C.uint64_t
	var st C.ngpu_layer_stats
	var info C.ngpu_blob_info
	rc := C.ngpu_pack_finish(w.p, nil, nil, nil, &pc, &pr, &n, &st, &info)
	w.pw.Close()
	w.done()
	if err := <-w.copied; err != nil && rc == 0 {
		return "", err
	}
	if rc != 0 {
		return "", errOf(w.g.e, rc, "pack close")
	}
	C.ngpu_free_host(unsafe.Pointer(pc))
	C.ngpu_free_host(unsafe.Pointer(pr))
	sum := C.GoBytes(unsafe.Pointer(&info.stream_digest[0]), 32)
	return digest.NewDigestFromEncoded(digest.SHA256, hex.EncodeToString(sum)), nil
}

// Merge replaces tool.Merge (builder.go:220-294): bootstraps are the layers'
// image.boot entries (read with the reference's own UnpackEntry), digests the
// layers' Digest.Hex(), lowest layer first; parentBoot is ParentBootstrapPath's
// contents (nil = none), prefetch MergeOption.PrefetchPatterns.  Returns the
// merged bootstrap (the overlaid inode tree, RAFS v5 or v6 as the layers) and
// the blob ids.
func Merge(boots [][]byte, digests []string, dictBoot, parentBoot []byte, prefetch string) ([]byte, []string, error) {
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
	r, pw, _ := os.Pipe()
	var out bytes.Buffer
	done := make(chan struct{})
	go func() { io.Copy(&out, r); r.Close(); close(done) }()
	var ids *C.char
	rc := C.ngpu_merge_ex((*unsafe.Pointer)(ptrs), (*C.uint64_t)(sizes), (**C.char)(names),
		C.uint64_t(n), dict, C.uint64_t(len(dictBoot)), &mo, C.ngpu_write_fn(C.ngpu_write_fd),
		unsafe.Pointer(uintptr(pw.Fd())), &ids)
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
// device, Packs spread round robin, one chunk dict for all of them -- replicated on every GPU or
// partitioned by digest prefix with the probe exchange over xGMI inside the library.
type Node struct{ n *C.ngpu_node }

func NewNode(devices []int32, digester, chunkSize, fsVersion uint32) (*Node, error) {
	cfg := C.ngpu_config{digester: C.uint32_t(digester), chunk_size: C.uint32_t(chunkSize),
		fs_version: C.uint32_t(fsVersion)}
	var n *C.ngpu_node
	if rc := C.ngpu_node_create((*C.int32_t)(unsafe.Pointer(&devices[0])), C.uint32_t(len(devices)), &cfg, &n); rc != 0 {
		return nil, errOf(nil, rc, "node")
	}
	return &Node{n}, nil
}

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

// Engine i of the node, for Pack: `nd.Engine(i % n).Pack(ctx, dest, comp, dict)`.
func (nd *Node) Engine(i int) *Engine { return &Engine{C.ngpu_node_engine(nd.n, C.uint32_t(i))} }

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
