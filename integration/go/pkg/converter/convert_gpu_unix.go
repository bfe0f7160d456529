//go:build !windows
// +build !windows

// convert_gpu_unix.go — the GPU branch of converter.Pack / Merge / Unpack
// (pkg/converter/convert_unix.go:325-362, 560-666, 669-719): the chunk
// digest + dedup stage in-process on MI355X through pkg/gpu (libnydusgpu.so)
// instead of the `nydus-image` child process (tool.Pack / tool.Merge /
// tool.Unpack, pkg/converter/tool/builder.go:148-178, 220-362).
// ../../converter.patch adds the PackOption fields and the calls into this
// file; everything else in pkg/converter is unchanged.
//
// NOT COMPILED HERE: this container has no Go toolchain (SURVEY.md §8(c)).
// The same logic runs as the C++ mirror (nydus-snapshotter_amd/host/
// converter.cpp, tests/cpp/converter_test.cpp) and the Python mirror
// (nydus_gpu/converter.py, tests/test_gpu_rafs.py).

package converter

import (
	"bytes"
	"context"
	"fmt"
	"io"
	"os"
	"path/filepath"
	"strconv"
	"strings"
	"sync"

	"github.com/containerd/containerd/v2/core/content"
	"github.com/opencontainers/go-digest"
	"github.com/pkg/errors"

	"github.com/containerd/nydus-snapshotter/pkg/converter/tool"
	"github.com/containerd/nydus-snapshotter/pkg/gpu"
)

type gpuKey struct {
	digester, chunkSize, fsVersion, flags uint32
}

var (
	gpuMu    sync.Mutex
	gpuNodes = map[gpuKey]*gpu.Node{}
)

// gpuDevices: NYDUS_GPU_DEVICES ("0,1,2,3"; a device may repeat) or every
// device the library sees.
func gpuDevices() []int32 {
	var devs []int32
	if v := os.Getenv("NYDUS_GPU_DEVICES"); v != "" {
		for _, f := range strings.Split(v, ",") {
			if d, err := strconv.Atoi(strings.TrimSpace(f)); err == nil {
				devs = append(devs, int32(d))
			}
		}
	}
	if len(devs) == 0 {
		for i := 0; i < gpu.DeviceCount(); i++ {
			devs = append(devs, int32(i))
		}
	}
	return devs
}

// gpuNode returns the process's node for this option set: one engine per GPU
// of the host, each Pack on the least-loaded one, so the layers of an image --
// LayerConvertFunc runs one per goroutine (convert_unix.go:467-538) -- shard
// over every GPU and every GPU's PCIe link (north star: "the chunk stream is
// sharded by layer").
func gpuNode(opt PackOption) (*gpu.Node, error) {
	k := gpuKey{digester: gpu.Blake3, fsVersion: 6}
	if opt.Digester == "sha256" {
		k.digester = gpu.Sha256
	} else if opt.Digester != "" && opt.Digester != "blake3" {
		return nil, fmt.Errorf("invalid digester %q", opt.Digester)
	}
	if opt.FsVersion == "5" {
		k.fsVersion = 5
	}
	if opt.ChunkSize != "" {
		v, err := strconv.ParseUint(opt.ChunkSize, 0, 32) // "0x100000" as the CLI takes it
		if err != nil {
			return nil, errors.Wrap(err, "parse chunk size")
		}
		k.chunkSize = uint32(v) // the library enforces types.go:76's rule (NGPU_EINVAL)
	}
	if opt.AlignedChunk && k.fsVersion == 5 {
		k.flags |= gpu.AlignedChunk
	}
	gpuMu.Lock()
	defer gpuMu.Unlock()
	if nd, ok := gpuNodes[k]; ok {
		return nd, nil
	}
	nd, err := gpu.NewNode(gpuDevices(), k.digester, k.chunkSize, k.fsVersion, k.flags)
	if err != nil {
		return nil, err
	}
	gpuNodes[k] = nd
	return nd, nil
}

func compressorOf(name string) (uint32, error) {
	switch name {
	case "", "zstd":
		return CompressorZstd, nil
	case "none":
		return CompressorNone, nil
	case "lz4_block":
		return CompressorLz4Block, nil
	}
	return 0, fmt.Errorf("unsupported compressor %q", name)
}

// useGPU: the branch is taken only for what the library implements -- tar-rafs
// with no batch chunks and no encryption (the detected feature set decides,
// as it decides the builder's arguments); anything else keeps nydus-image.
func useGPU(opt PackOption) bool {
	if opt.Accelerator != "gpu" || !gpu.Available() {
		return false
	}
	if opt.features.Contains(tool.FeatureBatchSize) || opt.features.Contains(tool.FeatureEncrypt) {
		return false
	}
	return !opt.OCIRef || opt.FsVersion == "6"
}

// packGPU is Pack's GPU branch: a write-closer over gpu.PackWriter instead of
// packFromTar's FIFO + nydus-image pair (convert_unix.go:443-539).  Write
// takes the uncompressed layer tar (with OCIRef: the original gzip blob);
// Close writes the rest of the nydus stream to dest.
func packGPU(ctx context.Context, dest io.Writer, opt PackOption) (io.WriteCloser, error) {
	if opt.OCIRef { // packFromTar passes nothing but the blob for targz-ref (builder.go:180-218)
		opt = PackOption{Accelerator: opt.Accelerator, OCIRef: true, FsVersion: "6", Timeout: opt.Timeout}
	}
	nd, err := gpuNode(opt)
	if err != nil {
		return nil, errors.Wrap(err, "gpu node")
	}
	comp, err := compressorOf(opt.Compressor)
	if err != nil {
		return nil, err
	}
	// this Pack's own reference to a replica on every GPU of the node (a probe
	// needs no exchange); the library loads an unchanged ChunkDictPath once per node
	var dict *gpu.ChunkDict
	if opt.ChunkDictPath != "" && !opt.OCIRef {
		if dict, err = nd.OpenChunkDict(opt.ChunkDictPath, false); err != nil {
			return nil, errors.Wrap(err, "load chunk dict")
		}
		defer dict.Release() // the pack holds its own reference
	}
	cancel := context.CancelFunc(func() {})
	if opt.Timeout != nil { // builder.go:153-158
		ctx, cancel = context.WithTimeout(ctx, *opt.Timeout)
	}
	fsv := uint32(6)
	if opt.FsVersion == "5" {
		fsv = 5
	}
	pw, err := nd.Pack(ctx, dest, comp, fsv, opt.PrefetchPatterns, dict, opt.OCIRef)
	if err != nil {
		cancel()
		return nil, err
	}
	return &gpuPackWriter{pw: pw, cancel: cancel}, nil
}

// gpuPackWriter: the PackOption.Timeout context is cancelled on every end of
// the Pack (its AfterFunc then finds the pack already released), not only at
// Close, which LayerConvertFunc skips on its error paths.
type gpuPackWriter struct {
	pw     *gpu.PackWriter
	cancel context.CancelFunc
}

func (w *gpuPackWriter) Write(b []byte) (int, error) {
	n, err := w.pw.Write(b)
	if err != nil {
		w.cancel()
	}
	return n, err
}

func (w *gpuPackWriter) ReadFrom(r io.Reader) (int64, error) {
	n, err := w.pw.ReadFrom(r)
	if err != nil {
		w.cancel()
	}
	return n, err
}

func (w *gpuPackWriter) Close() error {
	defer w.cancel()
	_, err := w.pw.Close()
	return errors.Wrap(err, "convert nydus")
}

// mergeGPU replaces tool.Merge (builder.go:220-294) once Merge has unpacked
// every layer's bootstrap exactly as today (UnpackEntry over the layer's
// ReaderAt): the merged bootstrap goes to `target`, the referenced blob ids
// come back as digests, as tool.Merge builds them from its output JSON
// (builder.go:286-292).  rafs[l]: layer l's --blob-digests / --blob-sizes /
// --blob-toc-digests entry when it is a targz-ref layer (nil otherwise).
func mergeGPU(boots [][]byte, layerHexes []string, opt MergeOption, rafs []*gpu.RafsBlob,
	target io.Writer) ([]digest.Digest, error) {
	var dictBoot, parentBoot []byte
	var err error
	if opt.ChunkDictPath != "" {
		if dictBoot, err = os.ReadFile(opt.ChunkDictPath); err != nil {
			return nil, errors.Wrap(err, "read chunk dict")
		}
	}
	if opt.ParentBootstrapPath != "" {
		if parentBoot, err = os.ReadFile(opt.ParentBootstrapPath); err != nil {
			return nil, errors.Wrap(err, "read parent bootstrap")
		}
	}
	merged, ids, err := gpu.Merge(boots, layerHexes, dictBoot, parentBoot, opt.PrefetchPatterns, rafs)
	if err != nil {
		return nil, errors.Wrap(err, "merge bootstrap")
	}
	if _, err := io.Copy(target, bytes.NewReader(merged)); err != nil {
		return nil, err
	}
	out := make([]digest.Digest, 0, len(ids))
	for _, id := range ids {
		if id != "" {
			out = append(out, digest.NewDigestFromEncoded(digest.SHA256, id))
		}
	}
	return out, nil
}

// mergeGPUFiles is Merge's call site of mergeGPU: the layers' bootstraps as
// Merge unpacked them (sourceBootstrapPaths), their file names as the layer
// names -- Digest.Hex(), or OriginalDigest.Hex() for a targz-ref layer
// (getBootstrapPath, convert_unix.go:567-573), the names nydus-image merge
// sees -- the merged bootstrap written to target.  rafsBlobDigests / Sizes /
// TOCDigests are Merge's lists as it builds them for tool.Merge
// (convert_unix.go:577-590): one entry per layer with an OriginalDigest, in
// layer order.
func mergeGPUFiles(paths []string, layers []Layer, opt MergeOption, target string,
	rafsBlobDigests []string, rafsBlobSizes []int64, rafsBlobTOCDigests []string) ([]digest.Digest, error) {
	boots := make([][]byte, len(paths))
	hexes := make([]string, len(paths))
	var rafs []*gpu.RafsBlob
	j := 0
	for i, p := range paths {
		b, err := os.ReadFile(p)
		if err != nil {
			return nil, errors.Wrap(err, "read source bootstrap")
		}
		boots[i], hexes[i] = b, filepath.Base(p)
		if layers[i].OriginalDigest != nil {
			if j >= len(rafsBlobDigests) || j >= len(rafsBlobSizes) || j >= len(rafsBlobTOCDigests) {
				return nil, fmt.Errorf("targz-ref layer %d without its RAFS blob entry", i)
			}
			if rafs == nil {
				rafs = make([]*gpu.RafsBlob, len(paths))
			}
			rafs[i] = &gpu.RafsBlob{Digest: rafsBlobDigests[j], Size: rafsBlobSizes[j],
				TOCDigest: rafsBlobTOCDigests[j]}
			j++
		}
	}
	f, err := os.Create(target)
	if err != nil {
		return nil, errors.Wrap(err, "create target bootstrap")
	}
	defer f.Close()
	return mergeGPU(boots, hexes, opt, rafs, f)
}

// unpackGPU replaces unpackNydusBlob + tool.Unpack (convert_unix.go:669-719)
// for a non-streaming Unpack: the nydus stream is read once and written back
// as the OCI tar.
func unpackGPU(ra content.ReaderAt, dest io.Writer) error {
	stream := make([]byte, ra.Size())
	if _, err := ra.ReadAt(stream, 0); err != nil && err != io.EOF {
		return errors.Wrap(err, "read nydus stream")
	}
	return gpu.Unpack(stream, dest)
}
