"""FedOpt over client updates that do not fit in HBM at once (BASELINE.json configs[4]: 1 B-param
bf16 x 128 clients = 256 GB), streamed from host memory in waves, parameter-sliced over the
node's GPUs.

FEDn folds the pseudo-gradient client by client in queue order (fedopt.py:89-94) and applies the
server step once (fedopt.py:110-118). Here the K host-resident updates (pinned CPU tensors, one
flat buffer each, e.g. decoded by the streaming ingest) go to the devices W at a time: device d
copies ONLY its parameter slice [lo_d, hi_d) of every update over its own PCIe link (one copy
stream per device, two wave buffers: the H2D of wave i+1 overlaps the fold of wave i), folds the
wave into its slice of the running pseudo-gradient (``fa_fedopt_step`` without FINAL keeps pg in
HBM; FIRST on the first wave), and the last wave's launch also runs the server step on its slice
(FINAL) with its slices of old / m / v resident, so pg makes no last HBM round trip and no K = 0
launch follows (``fuse_final=False`` keeps the separate K = 0 FINAL launch, for A/B). Every element
sees the same client order and the same kernel arithmetic, so the result is bit-identical for any
device count, any wave size and either finish.
"""
import numpy as np
import torch

from . import ops, reuse
from .sharded import shard_bounds


class WaveFedOpt:
    """One session's FedOpt state sliced over ``devices`` (a list; a device may repeat, e.g. on a
    one-GPU box), for P-element flat models whose updates stream from host memory."""

    def __init__(self, devices, P, wave=8, fuse_final=True):
        self.devices = [torch.device(d) for d in devices]
        self.devices = [torch.device(d.type, torch.cuda.current_device()) if d.index is None else d
                        for d in self.devices]
        self.P = P
        self.wave = wave
        self.fuse_final = fuse_final
        self.bounds = shard_bounds(P, len(self.devices))
        self.m = [None] * len(self.devices)
        self.v = [None] * len(self.devices)
        self.copy = [torch.cuda.Stream(d) for d in self.devices]
        self.compute = [torch.cuda.current_stream(d) for d in self.devices]

    def round(self, host_updates, ns, old, params, kernel_times=None):
        """One aggregation round: ``host_updates`` = K flat CPU tensors (pinned for full-rate
        H2D) in FIFO order, ``ns`` their num_examples, ``old`` the global model as one flat
        tensor per device slice (``old[d]`` on device d, any dtype fa_fedopt_step takes).
        Returns the new model as per-device f64 slices; m / v stay on the devices.
        ``kernel_times``: a dict to receive, per launch kind ("first" wave, later "mid" waves, the
        last wave with the server step fused, "mid_final" or "first_final" when it is the only one;
        "final", the K = 0 server step, with ``fuse_final=False``), the list of (device, elements,
        clients, ms) of every launch (HIP events on the launch stream) — bench.py's per-kernel
        rooflines."""
        K = len(host_updates)
        if K == 0:
            raise ValueError("no updates")
        if len(ns) != K:
            raise ValueError(f"{K} updates but {len(ns)} num_examples")
        upd_dt = host_updates[0].dtype
        for k, u in enumerate(host_updates):      # a copy_ into the wave slots would cast silently
            if u.dtype != upd_dt or u.numel() != self.P or u.device.type != "cpu":
                raise ValueError(f"update {k}: {u.dtype} x {u.numel()} on {u.device}; every update must be a "
                                 f"host tensor of {self.P} {upd_dt} elements")
        for d, (lo, hi) in enumerate(self.bounds):
            if old[d].numel() != hi - lo or old[d].device != self.devices[d]:
                raise ValueError(f"old[{d}] must hold the {hi - lo} elements of slice {d} on {self.devices[d]}")
        Ns = [int(v) for v in np.cumsum(ns)]
        W = self.wave
        outs = []
        ctx = []
        for d, dv in enumerate(self.devices):
            lo, hi = self.bounds[d]
            with torch.cuda.device(dv):
                n = hi - lo
                pg_dt, m_dt = ops.fedopt_dtypes(upd_dt, old[d].dtype, None if self.m[d] is None else self.m[d].dtype)
                slots = [[reuse.watch(torch.empty(n, dtype=upd_dt, device=dv)) for _ in range(min(W, K))]
                         for _ in range(2)]
                ctx.append({"n": n, "slots": slots, "pg": torch.empty(n, dtype=pg_dt, device=dv), "m_dt": m_dt,
                            "loaded": [torch.cuda.Event() for _ in range(2)],
                            "used": [torch.cuda.Event() for _ in range(2)]})
        waves = (K + W - 1) // W
        opt = dict(serveropt=params.get("serveropt", "adam"), learning_rate=params.get("learning_rate", 1e-3),
                   beta1=params.get("beta1", 0.9), beta2=params.get("beta2", 0.99), tau=params.get("tau", 1e-4))
        for d, dv in enumerate(self.devices):
            c = ctx[d]
            with torch.cuda.device(dv):
                c["m_out"] = torch.empty(c["n"], dtype=c["m_dt"], device=dv)
                c["v_out"] = self.v[d] if self.v[d] is not None else torch.empty(c["n"], dtype=torch.float64, device=dv)
                c["out"] = torch.empty(c["n"], dtype=torch.float64, device=dv)
                # the slots' HBM came from the compute stream's pool: its previous owners' queued work
                # there runs before the copy stream's first H2D overwrites it
                self.copy[d].wait_stream(self.compute[d])
        for w in range(waves):                       # every device's wave w, then wave w + 1, ...
            b = w % 2
            ks = list(range(w * W, min(K, (w + 1) * W)))
            last = self.fuse_final and w == waves - 1
            for d, dv in enumerate(self.devices):
                lo, hi = self.bounds[d]
                c = ctx[d]
                if c["n"] == 0:
                    continue
                with torch.cuda.device(dv):
                    if w >= 2:
                        self.copy[d].wait_event(c["used"][b])     # the fold of wave w-2 read these buffers
                    with torch.cuda.stream(self.copy[d]):
                        for j, k in enumerate(ks):
                            c["slots"][b][j].copy_(host_updates[k][lo:hi], non_blocking=True)
                        c["loaded"][b].record(self.copy[d])
                    self.compute[d].wait_event(c["loaded"][b])
                    ev = self._span(kernel_times, d)
                    if last:                                  # the last wave folds and steps in one launch
                        ops.fedopt_step(old[d], c["slots"][b][:len(ks)], [ns[k] for k in ks], [Ns[k] for k in ks],
                                        first=(w == 0), final=True, pg=c["pg"], m_in=self.m[d], m_out=c["m_out"],
                                        v_in=self.v[d], v_out=c["v_out"], out=c["out"], stream=self.compute[d], **opt)
                    else:
                        ops.fedopt_step(old[d], c["slots"][b][:len(ks)], [ns[k] for k in ks], [Ns[k] for k in ks],
                                        first=(w == 0), final=False, pg=c["pg"], stream=self.compute[d])
                    self._end(kernel_times, ("first" if w == 0 else "mid") + ("_final" if last else ""), d, ev,
                              c["n"], len(ks))
                    c["used"][b].record(self.compute[d])
        for d, dv in enumerate(self.devices):
            c = ctx[d]
            with torch.cuda.device(dv):
                if c["n"] and not self.fuse_final:
                    ev = self._span(kernel_times, d)
                    ops.fedopt_step(old[d], [], [], [], first=False, final=True, pg=c["pg"], m_in=self.m[d],
                                    m_out=c["m_out"], v_in=self.v[d], v_out=c["v_out"], out=c["out"],
                                    stream=self.compute[d], upd_dtype=upd_dt, **opt)
                    self._end(kernel_times, "final", d, ev, c["n"], 0)
                self.m[d], self.v[d] = c["m_out"], c["v_out"]
                outs.append(c["out"])
        for d, dv in enumerate(self.devices):
            torch.cuda.synchronize(dv)
        if kernel_times is not None:
            for kind, spans in list(kernel_times.items()):
                kernel_times[kind] = [(d, n, k, a.elapsed_time(b)) for d, n, k, a, b in spans]
        return outs

    def _span(self, kernel_times, d):
        if kernel_times is None:
            return None
        a = torch.cuda.Event(enable_timing=True)
        a.record(self.compute[d])
        return a

    def _end(self, kernel_times, kind, d, a, n, k):
        if kernel_times is None:
            return
        b = torch.cuda.Event(enable_timing=True)
        b.record(self.compute[d])
        kernel_times.setdefault(kind, []).append((d, n, k, a, b))

    def slices(self, flat):
        """``flat`` (a host or device tensor of P elements) cut into per-device slices on their devices."""
        return [flat[lo:hi].to(dv) for (lo, hi), dv in zip(self.bounds, self.devices)]

    def gather(self, per_dev):
        """Per-device slices -> one host tensor (each device copies its slice over its own link)."""
        host = torch.empty(self.P, dtype=per_dev[0].dtype, pin_memory=True)
        for (lo, hi), t, dv in zip(self.bounds, per_dev, self.devices):
            with torch.cuda.device(dv):
                host[lo:hi].copy_(t, non_blocking=True)
        for dv in self.devices:
            torch.cuda.synchronize(dv)
        return host
