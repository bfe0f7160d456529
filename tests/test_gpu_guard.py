"""The unwritten-digest guard (VERDICT r2 "What's weak" 1): a chunk that
reaches the dedup stage without a digest written by this call's digest kernels
must fail the call, never come back as a plausible NEW / INTRA record.

The digest stage stores kind = NGPU_DIGESTED next to every digest; the dedup
stage takes only records marked so with a non-zero digest, marks any other
NGPU_UNHASHED (no dedup decision, not in the layered dict), and the call fails
with NGPU_EDEVICE naming the first such chunk.  Calls that read no stats leave
the error for ngpu_device_status.  Each test forces an unwritten slot through
the product ABI (split stages: digest, then clobber one record on the device,
then dedup) on each dedup path: the single-layer LDS stage, the multi-layer
one-workgroup stage and the grid kernels."""
import numpy as np
import pytest

import nydus_gpu

pytestmark = pytest.mark.gpu


def _layer(rng, n, size):
    data = rng.integers(0, 256, n * size, dtype=np.uint8)
    # chunks 0 and 5 equal (INTRA pair), chunk 7 equal to the clobbered chunk 3
    data[5 * size:6 * size] = data[0:size]
    data[7 * size:8 * size] = data[3 * size:4 * size]
    ch = np.zeros(n, nydus_gpu.CHUNK_DTYPE)
    ch["offset"] = np.arange(n) * size
    ch["length"] = size
    return data, ch


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()


PATHS = [("lds", 0, 1), ("grid", nydus_gpu.FLAG_GRID_STAGES, 1), ("layers", 0, 2)]


@pytest.mark.parametrize("path,flags,layers", PATHS, ids=[p[0] for p in PATHS])
@pytest.mark.parametrize("clobber", ["kind", "zero_digest"])
def test_unwritten_digest_fails_the_call(path, flags, layers, clobber, oracle):
    import torch
    rng = np.random.default_rng(7)
    n, size = 64, 4096
    data, ch = _layer(rng, n, size)
    eng = nydus_gpu.Engine(chunk_size=0x10000, flags=flags)
    try:
        d_data, d_ch = _dev(data), _dev(ch)
        out = torch.zeros(n * 64, dtype=torch.uint8, device="cuda")
        eng.digest_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), n, out.data_ptr())
        torch.cuda.synchronize()
        rec = out.view(n, 64)
        assert (rec[:, 32:36].cpu().numpy().view(np.uint32)[:, 0] == nydus_gpu.DIGESTED).all()
        j = 3
        if clobber == "kind":  # a record the digest stage never reached (stale kind)
            rec[j, 32:36] = 0
        else:  # the record of the r2 failure: kind written, digest all zero
            rec[j, 0:32] = 0
        torch.cuda.synchronize()
        if layers == 1:
            with pytest.raises(nydus_gpu.NgpuError) as ei:
                eng.dedup_device(d_ch.data_ptr(), n, out.data_ptr(), want_stats=True)
            assert ei.value.code == nydus_gpu.EDEVICE
            assert "first chunk 3" in str(ei.value), str(ei.value)
            with pytest.raises(nydus_gpu.NgpuError) as ei2:
                eng.device_status()
            assert ei2.value.code == nydus_gpu.EDEVICE
        else:  # device stats, no host read: only ngpu_device_status reports it
            first = torch.tensor([0, n // 2, n], dtype=torch.int64, device="cuda")
            st = torch.zeros(layers * 56, dtype=torch.uint8, device="cuda")
            eng.dedup_layers_device(d_ch.data_ptr(), n, out.data_ptr(), first.data_ptr(), layers,
                                    st.data_ptr())
            with pytest.raises(nydus_gpu.NgpuError) as ei:
                eng.device_status()
            assert ei.value.code == nydus_gpu.EDEVICE and "first chunk 3" in str(ei.value)
        eng.device_status()  # cleared by the check
        got = out.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
        assert got["kind"][j] == nydus_gpu.UNHASHED and got["index"][j] == 0xFFFFFFFF
        # chunk 7 (same bytes as 3) must not resolve INTRA to the unhashed chunk
        assert got["kind"][7] == nydus_gpu.NEW
        assert got["kind"][5] == nydus_gpu.INTRA and got["ref"][5] == 0
        others = np.ones(n, bool)
        others[j] = False
        assert (got["kind"][others] <= nydus_gpu.DICT).all()
    finally:
        eng.close()


def test_clean_calls_leave_no_device_error():
    import torch
    rng = np.random.default_rng(8)
    data, ch = _layer(rng, 32, 8192)
    eng = nydus_gpu.Engine(chunk_size=0x10000)
    try:
        d_data, d_ch = _dev(data), _dev(ch)
        out = torch.zeros(32 * 64, dtype=torch.uint8, device="cuda")
        for _ in range(3):
            eng.process_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), 32, out.data_ptr())
        eng.device_status()
        st = eng.process_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), 32,
                                out.data_ptr(), want_stats=True)
        assert st["intra_chunks"] == 2
    finally:
        eng.close()


def test_stale_records_from_a_previous_call_are_caught():
    """Dedup twice over the same records: the second call sees the first
    call's NEW / INTRA records, not digest-stage output, and must fail."""
    import torch
    rng = np.random.default_rng(9)
    data, ch = _layer(rng, 16, 4096)
    eng = nydus_gpu.Engine(chunk_size=0x10000)
    try:
        d_data, d_ch = _dev(data), _dev(ch)
        out = torch.zeros(16 * 64, dtype=torch.uint8, device="cuda")
        eng.process_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), 16, out.data_ptr(),
                           want_stats=True)
        with pytest.raises(nydus_gpu.NgpuError) as ei:
            eng.dedup_device(d_ch.data_ptr(), 16, out.data_ptr(), want_stats=True)
        assert ei.value.code == nydus_gpu.EDEVICE and "16 chunk(s)" in str(ei.value)
        with pytest.raises(nydus_gpu.NgpuError):
            eng.device_status()
    finally:
        eng.close()


def test_bad_descriptor_reported_by_device_status():
    """device entry points without host stats surface bad /
    overlapping descriptors through ngpu_device_status."""
    import torch
    rng = np.random.default_rng(10)
    data, ch = _layer(rng, 8, 4096)
    ch["offset"][2] = len(data)  # past the buffer
    eng = nydus_gpu.Engine(chunk_size=0x10000)
    try:
        d_data, d_ch = _dev(data), _dev(ch)
        out = torch.zeros(8 * 64, dtype=torch.uint8, device="cuda")
        eng.process_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), 8, out.data_ptr())
        with pytest.raises(nydus_gpu.NgpuError) as ei:
            eng.device_status()
        assert ei.value.code == nydus_gpu.EINVAL and "outside" in str(ei.value)
        eng.device_status()
    finally:
        eng.close()


def test_first_call_of_fresh_engines_on_nonblocking_streams(oracle):
    """The round-2 zero digest, root-caused in round 4: an engine's first call
    zeroed its new stats words with hipMemset, which is asynchronous to the
    host and runs on the null stream -- unordered with a caller's
    non-blocking stream.  Landing after the first digest kernel wrote its
    counters and before b3_tree read them, it zeroed the tree queue count and
    the multi-leaf chunks kept no digest (tools/step_diag.py reproduced it on
    2 of 3 first node steps over 8 streams).  Here the null stream is kept
    busy by a fill of a different length before each fresh engine's first
    call on its own non-blocking stream, so a queued memset lands at a
    different point of that call's digest each time: every digest must equal
    the oracle's and no guard may fire.  (On this pool the pre-fix build
    passes this test too -- the null stream and a caller's stream may share a
    hardware queue, which orders them; the reproducer is the first 8-stream
    node step, test_gpu_node.py::test_node_step_all_devices_at_once_vs_oracle[8]
    and scripts/gpu_race_ab.sh.)"""
    import torch
    rng = np.random.default_rng(2024)
    cs = 0x10000
    total = 24 << 20  # quad path, planning in the leaf kernel: b3_tree reads the queue count
    data = rng.integers(0, 256, total, dtype=np.uint8)
    ch = np.zeros(total // cs, nydus_gpu.CHUNK_DTYPE)
    ch["offset"] = np.arange(len(ch)) * cs
    ch["length"] = cs
    ch["length"][::7] = rng.integers(1, cs, len(ch[::7]))
    ch["file_index"] = np.arange(len(ch))
    dig = oracle.digest_chunks(data.tobytes(), ch.view(oracle.CHUNK_DTYPE), "blake3")
    d_data = torch.from_numpy(data).cuda()
    d_ch = torch.from_numpy(ch.view(np.uint8).copy()).cuda()
    big = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")
    assert torch.cuda.current_stream().cuda_stream == 0  # fills go to the null stream
    fills = [0] + [(1 << 20) << k for k in range(12)]  # 0, 1 MiB .. 2 GiB
    engines, outs, streams = [], [], []
    try:
        for _ in fills:
            engines.append(nydus_gpu.Engine(device=0, chunk_size=cs))
            outs.append(torch.zeros(len(ch) * 64, dtype=torch.uint8, device="cuda"))
            streams.append(torch.cuda.Stream())
        torch.cuda.synchronize()
        for e, o, s, f in zip(engines, outs, streams, fills):
            if f:
                big[:f].fill_(f & 0xFF)  # null stream busy for ~f / 4 TB/s
            e.process_device(d_data.data_ptr(), d_data.numel(), d_ch.data_ptr(), len(ch), o.data_ptr(),
                             stream=s.cuda_stream)
        torch.cuda.synchronize()
        for k, (e, o) in enumerate(zip(engines, outs)):
            got = o.cpu().numpy().view(nydus_gpu.RESULT_DTYPE)
            assert np.array_equal(got["digest"], dig), (k, fills[k])
            e.device_status()
    finally:
        for e in engines:
            e.close()
