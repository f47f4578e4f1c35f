"""Runs the product (librazor_fec.so, HIP kernels) on numpy inputs: uploads to
HBM with torch (allocator only), calls the C ABI, downloads the results."""
from __future__ import annotations

import numpy as np
import torch

from razor_amd.fec import HDR_DTYPE, native


def _dev(a: np.ndarray, device) -> torch.Tensor:
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to(device)


def _host(t: torch.Tensor, dtype, shape) -> np.ndarray:
    return t.cpu().numpy().view(dtype).reshape(shape)


class GpuEngine:
    def __init__(self, video_size=1000, device="cuda:0", tuning=0, random_workspace=False):
        self.lib = native(video_size)
        self.device = torch.device(device)
        self.tuning = tuning
        self.random_workspace = random_workspace  # recover workspace starts as random bytes (not zeroed)

    def encode(self, plan, shards, hdr, capacity):
        G, k, stride = shards.shape
        n = plan.n_lines
        d_sh = _dev(shards, self.device)
        d_h = _dev(hdr, self.device)
        d_p = torch.full((G * n * stride,), 0x5A, dtype=torch.uint8, device=self.device)
        d_m = torch.full((G * n * 20,), 0x5A, dtype=torch.uint8, device=self.device)
        d_f = torch.zeros((G * n,), dtype=torch.int16, device=self.device)
        d_s = torch.full((G * n,), 7, dtype=torch.int8, device=self.device)
        self.lib.set_tuning(self.tuning)
        try:
            self.lib.encode_batch(plan, G, stride, capacity, d_sh.data_ptr(), d_h.data_ptr(), d_p.data_ptr(),
                                  d_m.data_ptr(), d_f.data_ptr(), d_s.data_ptr(),
                                  torch.cuda.current_stream(self.device).cuda_stream)
            torch.cuda.synchronize(self.device)
        finally:
            self.lib.set_tuning(0)
        return (_host(d_p, np.uint8, (G, n, stride)), _host(d_m, HDR_DTYPE, (G, n)),
                _host(d_f, np.uint16, (G, n)), _host(d_s, np.int8, (G, n)))

    def recover(self, plan, shards, hdr, present, parity, meta, fsize, pp, capacity):
        G, k, stride = shards.shape
        d_sh = _dev(shards, self.device)
        d_h = _dev(hdr, self.device)
        d_pr = _dev(np.ascontiguousarray(present, np.uint64), self.device)
        d_p = _dev(parity, self.device)
        d_m = _dev(meta, self.device)
        d_f = _dev(np.ascontiguousarray(fsize, np.uint16), self.device)
        d_pp = _dev(np.ascontiguousarray(pp, np.uint64), self.device)
        d_rec = torch.full((G * 16,), 0xEE, dtype=torch.uint8, device=self.device)
        nws = max(16, self.lib.workspace_size(plan, G))
        ws = (torch.randint(0, 256, (nws,), dtype=torch.uint8, device=self.device) if self.random_workspace
              else torch.zeros((nws,), dtype=torch.uint8, device=self.device))
        self.lib.set_tuning(self.tuning)
        try:
            self.lib.recover_batch(plan, G, stride, capacity, d_sh.data_ptr(), d_h.data_ptr(), d_pr.data_ptr(),
                                   d_p.data_ptr(), d_m.data_ptr(), d_f.data_ptr(), d_pp.data_ptr(),
                                   d_rec.data_ptr(), ws.data_ptr(),
                                   torch.cuda.current_stream(self.device).cuda_stream)
            torch.cuda.synchronize(self.device)
        finally:
            self.lib.set_tuning(0)
        return (_host(d_sh, np.uint8, (G, k, stride)), _host(d_h, HDR_DTYPE, (G, k)),
                _host(d_rec, np.uint64, (G, 2)))

    def recover_out(self, plan, shards, hdr, present, parity, meta, fsize, pp, capacity, per_group):
        """rfec_recover_batch_out: returns (out_shards [G][E][stride], out_hdr
        [G][E], out_index [G][E], recovered [G][2]) and checks that the inputs
        were left untouched."""
        G, k, stride = shards.shape
        E = per_group
        d_sh = _dev(shards, self.device)
        d_h = _dev(hdr, self.device)
        d_pr = _dev(np.ascontiguousarray(present, np.uint64), self.device)
        d_p = _dev(parity, self.device)
        d_m = _dev(meta, self.device)
        d_f = _dev(np.ascontiguousarray(fsize, np.uint16), self.device)
        d_pp = _dev(np.ascontiguousarray(pp, np.uint64), self.device)
        d_rec = torch.full((G * 16,), 0xEE, dtype=torch.uint8, device=self.device)
        o_sh = torch.full((G * E * stride,), 0x3C, dtype=torch.uint8, device=self.device)
        o_h = torch.full((G * E * 20,), 0x3C, dtype=torch.uint8, device=self.device)
        o_i = torch.full((G * E,), 0x3C, dtype=torch.uint8, device=self.device)
        nws = max(16, self.lib.workspace_size(plan, G))
        ws = (torch.randint(0, 256, (nws,), dtype=torch.uint8, device=self.device) if self.random_workspace
              else torch.zeros((nws,), dtype=torch.uint8, device=self.device))
        self.lib.set_tuning(self.tuning)
        try:
            self.lib.recover_batch_out(plan, G, stride, capacity, d_sh.data_ptr(), d_h.data_ptr(), d_pr.data_ptr(),
                                       d_p.data_ptr(), d_m.data_ptr(), d_f.data_ptr(), d_pp.data_ptr(),
                                       d_rec.data_ptr(), E, o_sh.data_ptr(), o_h.data_ptr(), o_i.data_ptr(),
                                       ws.data_ptr(), torch.cuda.current_stream(self.device).cuda_stream)
            torch.cuda.synchronize(self.device)
        finally:
            self.lib.set_tuning(0)
        assert np.array_equal(_host(d_sh, np.uint8, (G, k, stride)), shards), "shards written"
        assert np.array_equal(_host(d_h, HDR_DTYPE, (G, k)), hdr), "headers written"
        return (_host(o_sh, np.uint8, (G, E, stride)), _host(o_h, HDR_DTYPE, (G, E)), _host(o_i, np.uint8, (G, E)),
                _host(d_rec, np.uint64, (G, 2)))


    def recover_packed(self, plan, shards, hdr, present, parity, meta, fsize, pp, capacity, per_group, packed=None):
        """rfec_pack_erasures (on the device, unless `packed` gives the records)
        then rfec_recover_packed_out: returns (out_shards, out_hdr, out_index,
        recovered, packed records [G][stride] as built)."""
        G, k, stride = shards.shape
        E = per_group
        pks = self.lib.packed_stride(plan, E)
        assert pks > 0
        st = torch.cuda.current_stream(self.device).cuda_stream
        d_sh = _dev(shards, self.device)
        d_p = _dev(parity, self.device)
        if packed is None:
            d_h = _dev(hdr, self.device)
            d_pr = _dev(np.ascontiguousarray(present, np.uint64), self.device)
            d_m = _dev(meta, self.device)
            d_f = _dev(np.ascontiguousarray(fsize, np.uint16), self.device)
            d_pp = _dev(np.ascontiguousarray(pp, np.uint64), self.device)
            d_pk = torch.full((G * pks,), 0x77, dtype=torch.uint8, device=self.device)
            self.lib.pack_erasures(plan, G, d_h.data_ptr(), d_pr.data_ptr(), d_m.data_ptr(), d_f.data_ptr(),
                                   d_pp.data_ptr(), E, d_pk.data_ptr(), st)
        else:
            assert packed.shape == (G, pks)
            d_pk = _dev(packed, self.device)
        d_rec = torch.full((G * 16,), 0xEE, dtype=torch.uint8, device=self.device)
        o_sh = torch.full((G * E * stride,), 0x3C, dtype=torch.uint8, device=self.device)
        o_h = torch.full((G * E * 20,), 0x3C, dtype=torch.uint8, device=self.device)
        o_i = torch.full((G * E,), 0x3C, dtype=torch.uint8, device=self.device)
        self.lib.recover_packed_out(plan, G, stride, capacity, d_sh.data_ptr(), d_p.data_ptr(), d_pk.data_ptr(),
                                    d_rec.data_ptr(), E, o_sh.data_ptr(), o_h.data_ptr(), o_i.data_ptr(), st)
        torch.cuda.synchronize(self.device)
        assert np.array_equal(_host(d_sh, np.uint8, (G, k, stride)), shards), "shards written"
        return (_host(o_sh, np.uint8, (G, E, stride)), _host(o_h, HDR_DTYPE, (G, E)), _host(o_i, np.uint8, (G, E)),
                _host(d_rec, np.uint64, (G, 2)), _host(d_pk, np.uint8, (G, pks)))


class GpuWire:
    """The wire codec (rfec_wire_*) on numpy inputs."""

    def __init__(self, video_size=1000, device="cuda:0", tuning=0):
        self.lib = native(video_size)
        self.device = torch.device(device)
        self.tuning = tuning  # RFEC_TUNE_WAVE_PARSE: the wave-per-datagram parse

    def _run(self, fn, *args):
        fn(*args, torch.cuda.current_stream(self.device).cuda_stream)
        torch.cuda.synchronize(self.device)

    def frame_fec(self, parity, meta, fsize, status, stamps, capacity, dstride):
        N, stride = parity.shape[0] if parity.ndim == 2 else parity.size // parity.shape[-1], parity.shape[-1]
        d_p, d_m, d_f, d_s = (_dev(a, self.device) for a in (parity, meta, np.ascontiguousarray(fsize, np.uint16),
                                                                stamps))
        d_st = None if status is None else _dev(np.ascontiguousarray(status, np.int8), self.device)
        d_g = torch.full((N * dstride,), 0xEE, dtype=torch.uint8, device=self.device)
        d_l = torch.full((N,), 0x7777, dtype=torch.int16, device=self.device)
        self._run(self.lib.wire_frame_fec, N, stride, capacity, d_p.data_ptr(), d_m.data_ptr(), d_f.data_ptr(),
                  None if d_st is None else d_st.data_ptr(), d_s.data_ptr(), dstride, d_g.data_ptr(), d_l.data_ptr())
        return _host(d_g, np.uint8, (N, dstride)), _host(d_l, np.uint16, (N,))

    def frame_seg(self, shards, hdr, stamps, capacity, dstride, order=None):
        stride = shards.shape[-1]
        N = shards.size // stride
        d_d, d_h, d_s = (_dev(a, self.device) for a in (shards, hdr, stamps))
        d_o = None if order is None else _dev(np.ascontiguousarray(order, np.uint32), self.device)
        d_g = torch.full((N * dstride,), 0xEE, dtype=torch.uint8, device=self.device)
        d_l = torch.full((N,), 0x7777, dtype=torch.int16, device=self.device)
        fn = lambda *a: self.lib.wire_frame_seg(*a, order=None if d_o is None else d_o.data_ptr())  # noqa: E731
        self._run(fn, N, stride, capacity, d_d.data_ptr(), d_h.data_ptr(), d_s.data_ptr(), dstride, d_g.data_ptr(),
                  d_l.data_ptr())
        return _host(d_g, np.uint8, (N, dstride)), _host(d_l, np.uint16, (N,))

    def parse(self, dgram, dlen, stride, capacity):
        N, dstride = dgram.shape
        d_g = _dev(dgram, self.device)
        d_l = _dev(np.ascontiguousarray(dlen, np.uint16), self.device)
        d_r = torch.full((N * 64,), 0xEE, dtype=torch.uint8, device=self.device)
        d_p = torch.full((N * stride,), 0xEE, dtype=torch.uint8, device=self.device)
        self.lib.set_tuning(self.tuning)
        try:
            self._run(self.lib.wire_parse, N, dstride, d_g.data_ptr(), d_l.data_ptr(), stride, capacity,
                      d_r.data_ptr(), d_p.data_ptr())
        finally:
            self.lib.set_tuning(0)
        from razor_amd.fec import WIRE_REC_DTYPE
        return _host(d_r, WIRE_REC_DTYPE, (N,)), _host(d_p, np.uint8, (N, stride))
