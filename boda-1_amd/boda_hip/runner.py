"""Per-op workload runner: the Python twin of ops-prof's profile_rcg_call
(src/rtc_prof.cc:44-126) over the C-ABI, used by bench.py and the GPU tests.

For each op: create its vars on the device (zero-filled), fill the inputs with
the reference's gen_data (mode 5 by default) on the device, then launch the
main kernel as often as asked, timing each launch between a pair of HIP
events on the context's stream (the reference times exactly this: one
main-kernel call, no data generation or layout transforms, F7: the filter-bank
transform the k-major conv kernels read is made once per op at setup, like the
reference's xpose_filts). A step can be
captured into a hipGraph and replayed, so the GPU runs the op sweep back to
back instead of waiting on per-launch host latency.
"""
from dataclasses import dataclass

from . import GEN_CONV_BIASES, GEN_CONV_FILTS, GEN_CONV_IN, GEN_SGEMM_A, GEN_SGEMM_B, conv_filts_packed_floats
from .ops import ConvShape, SgemmShape

# MI355X peaks (MI355X_MICROARCH.md): fp32 matrix = vector = 157.3 TFLOP/s; HBM3E 8.0 TB/s.
PEAK_FP32_FLOPS = 157.3e12
PEAK_HBM_BPS = 8.0e12


def roofline_secs(shape):
    """Per-op roofline time: max(flops / fp32 peak, algorithmic bytes / HBM peak)."""
    return max(shape.flops() / PEAK_FP32_FLOPS, shape.bytes() / PEAK_HBM_BPS)


def bound_of(shape):
    return "mfma" if shape.flops() / PEAK_FP32_FLOPS >= shape.bytes() / PEAK_HBM_BPS else "hbm"


@dataclass
class OpVars:
    shape: object
    bufs: tuple
    tag: str = ""


class Workload:
    def __init__(self, dev, shapes, mode=5, tags=None, pack=True):
        self.dev = dev
        self.ops = []
        for i, s in enumerate(shapes):
            tag = tags[i] if tags else ""
            if isinstance(s, SgemmShape):
                a = dev.alloc_floats(s.K * s.M)
                b = dev.alloc_floats(s.K * s.N)
                c = dev.alloc_floats(s.M * s.N)
                dev.gen_data(GEN_SGEMM_A, a, [s.K, s.M], mode)
                dev.gen_data(GEN_SGEMM_B, b, [s.K, s.N], mode)
                self.ops.append(OpVars(s, (a, b, c), tag))
            elif isinstance(s, ConvShape):
                inp = dev.alloc_floats(s.B * s.IC * s.H * s.W)
                f = dev.alloc_floats(s.OC * s.K)
                bi = dev.alloc_floats(s.OC)
                o = dev.alloc_floats(s.B * s.OC * s.OH * s.OW)
                dev.gen_data(GEN_CONV_IN, inp, [s.B, s.IC, s.H, s.W], mode)
                dev.gen_data(GEN_CONV_FILTS, f, [s.OC, s.IC, s.KY, s.KX], mode)
                dev.gen_data(GEN_CONV_BIASES, bi, [s.OC], mode)
                # the filter-bank transform, once per op before any timed call, as the
                # reference's xpose_filts (src/rtc_prof.cc:93-99; untimed, F7)
                pk = None
                if pack:
                    pk = dev.alloc_floats(conv_filts_packed_floats(s))
                    dev.conv_filts_pack(f, pk, s)
                self.ops.append(OpVars(s, (inp, f, bi, pk, o), tag))
            else:
                raise TypeError(s)
        dev.sync()

    def launch(self, i):
        v = self.ops[i]
        s = v.shape
        if isinstance(s, SgemmShape):
            a, b, c = v.bufs
            self.dev.sgemm(a, b, c, s.M, s.N, s.K)
        else:
            inp, f, bi, pk, o = v.bufs
            self.dev.conv(inp, f, bi, o, s, 1, packed=pk)

    def output(self, i):
        return self.ops[i].bufs[-1].download()

    def step(self, timed_events=None, stamp_base=None):
        """One pass over every op (one main-kernel launch each). With timed_events (a list),
        appends (op index, begin event, end event). With stamp_base, writes a device
        timestamp into slot stamp_base + i before op i and one after the last op, so op i
        took stamps[i+1] - stamps[i] (its kernel(s) plus one stamp and the launch seams)."""
        for i in range(len(self.ops)):
            if stamp_base is not None:
                self.dev.stamp(stamp_base + i)
            if timed_events is not None:
                b = self.dev.event()
                self.launch(i)
                e = self.dev.event()
                timed_events.append((i, b, e))
            else:
                self.launch(i)
        if stamp_base is not None:
            self.dev.stamp(stamp_base + len(self.ops))

    def step_kernel_timed(self, out):
        """One eager pass; each op's GPU time is recorded on its own first/last kernel
        dispatch (bh_time_next_call). Appends (op index, begin event, end event) to out."""
        for i in range(len(self.ops)):
            b, e = self.dev.time_next_call()
            self.launch(i)
            out.append((i, b, e))

    def op_graph_time(self, i, reps, spin_us=100):
        """Amortized GPU seconds per call of op i: `reps` back-to-back calls captured in
        one hipGraph and replayed behind a short spin kernel (so the whole batch is queued
        before the GPU reaches it), timed by HIP events recorded around the replay on the
        context's stream. This is the op's cost in a dense sweep (dispatch + run + drain),
        free of the ~2.5 us that events bound to each dispatch add to a lone call."""
        self.dev.capture_begin()
        try:
            for _ in range(reps):
                self.launch(i)
        finally:
            g = self.dev.capture_end()
        try:
            self.dev.graph_launch(g)  # warm: graph upload, caches, split-K workspaces
            self.dev.spin(spin_us)
            b = self.dev.event()
            self.dev.graph_launch(g)
            e = self.dev.event()
            self.dev.sync()
            return self.dev.elapsed_ms(b, e) / 1e3 / reps
        finally:
            self.dev.graph_destroy(g)

    def capture_step(self, stamp_base=None):
        """Capture one step into a hipGraph (HIP events cannot be timed inside graphs,
        so per-op times come from device stamps, see step()). Returns the graph id."""
        self.dev.capture_begin()
        try:
            self.step(stamp_base=stamp_base)
        finally:
            g = self.dev.capture_end()
        return g

    def free(self):
        for v in self.ops:
            for b in v.bufs:
                if b is not None:
                    b.free()
        self.ops = []
