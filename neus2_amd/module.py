"""tcnn-shaped operator modules over the gfx950 kernels (include/neus2_hip.h neus_module_*), mirroring
tiny-cuda-nn's C++ API (dependencies/my_tcnn/include/tiny-cuda-nn/cpp_api.h:66-110) the reference's bindings wrap:
create_network(n_input_dims, n_output_dims, network) / create_encoding / create_network_with_input_encoding (the names
mean what tcnn's mean) plus create_nerf_network (the NeuS NerfNetwork), n_params, initialize_params, inference, forward
(-> Context), backward, backward_backward_input with explicit parameter pointers and EGradientMode (object.h:90-94).

Arguments are torch CUDA tensors (device memory + the current stream); outputs are allocated here unless given.
"""
from __future__ import annotations

import ctypes as C
import enum
import json

from ._lib import NeusError, NeusModuleInfo, check, lib


class Precision(enum.IntEnum):  # tcnn::cpp::EPrecision (cpp_api.h:50-53)
    Fp32 = 0
    Fp16 = 1


class GradientMode(enum.IntEnum):
    Ignore = 0
    Overwrite = 1
    Accumulate = 2


def _p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream():
    import torch
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


class Context:
    def __init__(self, h, n):
        self._h, self.n = h, n

    def __del__(self):
        if getattr(self, "_h", None):
            lib().neus_context_destroy(self._h)
            self._h = None


class Module:
    """tcnn::cpp::Module. kind 'mlp' = create_network's Identity -> FullyFusedMLP (input [n, n_input_dims] f32, output
    [n, padded output] fp16), 'network' = the NeuS NerfNetwork (input [n, 7] f32, output [n, 16] fp16),
    'encoding' = the HashGrid encoding (input [n, 3] f32; output layout by the config's "output_layout": "AoS" [n, 2L]
    (default: the column-major view cpp::Module gives its caller, cpp_api.cu:58-70), "SoA" [2L, n] (GridEncoding's
    preferred layout, grid.h:2357-2359) or "paired" [L, n, 2] (this build's kernels)). dL_dparams is fp16 (tcnn's param
    precision) unless the config says "gradient_precision": "fp32"."""

    def __init__(self, handle, kind):
        self._h, self.kind = handle, kind
        info = NeusModuleInfo()
        check(lib().neus_module_info(self._h, C.byref(info)))
        self.info = {k: getattr(info, k) for k, _ in info._fields_}
        hp = self.hyperparams()
        self.output_layout = hp.get("output_layout", "AoS")
        self.gradient_precision = hp.get("gradient_precision", "fp16")
        self.precision = hp.get("precision", "fp16")

    @classmethod
    def create_network(cls, n_input_dims, n_output_dims, network, batch_capacity=1 << 18):
        """tcnn create_network (cpp_api.h:109; cpp_api.cu:170-172): NetworkWithInputEncoding with an Identity encoding and
        a FullyFusedMLP (`network`: {"otype": "FullyFusedMLP", "n_neurons", "n_hidden_layers", "activation",
        "output_activation"})."""
        text = network if isinstance(network, str) else json.dumps(network)
        h = C.c_void_p()
        check(lib().neus_module_create_network(C.c_uint32(n_input_dims), C.c_uint32(n_output_dims), text.encode(),
                                               C.c_uint32(batch_capacity), C.byref(h)))
        return cls(h, "mlp")

    @classmethod
    def create_nerf_network(cls, config, batch_capacity=1 << 18):
        """The NeuS NerfNetwork (nerf_network.h): `config` is the configs/nerf/*.json object (or its text) with
        "encoding", "network" and "rgb_network"."""
        text = config if isinstance(config, str) else json.dumps(config)
        h = C.c_void_p()
        check(lib().neus_module_create_nerf_network(text.encode(), C.c_uint32(batch_capacity), C.byref(h)))
        return cls(h, "network")

    @classmethod
    def create_network_with_input_encoding(cls, n_input_dims, n_output_dims, encoding, network, batch_capacity=1 << 18):
        """tcnn create_network_with_input_encoding (cpp_api.h:108; network_with_input_encoding.h): `encoding` HashGrid or
        Identity ({"scale", "offset"}, identity.h), `network` a FullyFusedMLP of any depth / width (16..128) / activation.
        Params [network matrices in order | grid] (network first, as NetworkWithInputEncoding's set_params_impl,
        network_with_input_encoding.h:262-270); output [n, padded n_output_dims] fp16; the grid's output is zero-padded to
        a multiple of 16 (grid.h:1540-1550). HashGrid -> one hidden ReLU layer with a linear output of <= 16 dims runs as
        the fused DensityNet kernel, anything else as the grid kernels feeding ffmlp.hip's MFMA layers;
        backward_backward_input as network_with_input_encoding.h:159-250."""
        te = encoding if isinstance(encoding, str) else json.dumps(encoding)
        tn = network if isinstance(network, str) else json.dumps(network)
        h = C.c_void_p()
        check(lib().neus_module_create_network_with_input_encoding(C.c_uint32(n_input_dims), C.c_uint32(n_output_dims), te.encode(),
                                                                   tn.encode(), C.c_uint32(batch_capacity), C.byref(h)))
        return cls(h, "network_with_input_encoding")

    @classmethod
    def create_encoding(cls, encoding, batch_capacity=1 << 18, n_input_dims=3, requested_precision=Precision.Fp16):
        """tcnn create_encoding(n_input_dims, encoding, requested_precision) (cpp_api.h:110; cpp_api.cu:174-180): Fp16 =
        GridEncoding<__half> (fp16 params / output), Fp32 = GridEncoding<float> (f32 params, output and gradients)."""
        text = encoding if isinstance(encoding, str) else json.dumps(encoding)
        h = C.c_void_p()
        check(lib().neus_module_create_encoding(C.c_uint32(n_input_dims), text.encode(), C.c_int(int(Precision(requested_precision))),
                                                C.c_uint32(batch_capacity), C.byref(h)))
        return cls(h, "encoding")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().neus_module_destroy(self._h)
            self._h = None

    @property
    def n_params(self):
        return int(self.info["n_params"])

    @property
    def n_input_dims(self):
        return int(self.info["n_input_dims"])

    @property
    def n_output_dims(self):
        return int(self.info["n_output_dims"])

    def hyperparams(self):
        n = C.c_uint64()
        check(lib().neus_module_hyperparams(self._h, None, C.c_uint64(0), C.byref(n)))
        buf = C.create_string_buffer(n.value + 1)
        check(lib().neus_module_hyperparams(self._h, buf, C.c_uint64(n.value + 1), None))
        return json.loads(buf.value.decode())

    def name(self):
        return self.hyperparams()["otype"]

    def set_training_step(self, step: int):
        check(lib().neus_module_set_training_step(self._h, C.c_int(int(step))))

    def set_indeed_batch_size(self, n: int):
        check(lib().neus_module_set_indeed_batch_size(self._h, C.c_uint32(int(n))))

    def initialize_params(self, seed=1337):
        import torch
        out = torch.empty(self.n_params, dtype=torch.float32, device="cuda")
        check(lib().neus_module_initialize_params(self._h, C.c_uint64(seed), _p(out)))
        return out

    def _out(self, n, output):
        import torch
        if output is not None:
            return output
        dt = torch.float32 if self.precision == "fp32" else torch.float16
        return torch.empty(self.output_shape(n), dtype=dt, device="cuda")

    def output_shape(self, n):
        if self.kind in ("mlp", "network_with_input_encoding"):
            return (n, self.n_output_dims)
        if self.kind != "encoding":
            return (n, 16)
        L = self.info["n_levels"]
        return {"AoS": (n, 2 * L), "SoA": (2 * L, n), "paired": (L, n, 2)}[self.output_layout]

    def gradient_buffer(self):
        """A zeroed dL_dparams tensor of the module's gradient precision."""
        import torch
        dt = torch.float16 if self.gradient_precision == "fp16" else torch.float32
        return torch.zeros(self.n_params, dtype=dt, device="cuda")

    def inference(self, x, params, output=None):
        n = x.shape[0]
        out = self._out(n, output)
        check(lib().neus_module_inference(self._h, _stream(), C.c_uint32(n), _p(x), _p(out), _p(params)))
        return out

    def forward(self, x, params, prepare_input_gradients=False, output=None):
        n = x.shape[0]
        out = self._out(n, output)
        h = C.c_void_p()
        check(lib().neus_module_forward(self._h, _stream(), C.c_uint32(n), _p(x), _p(out), _p(params),
                                        C.c_int(int(bool(prepare_input_gradients))), C.byref(h)))
        return Context(h, n), out

    def backward(self, ctx, x, dL_doutput, params, dL_dparams=None, dL_dinput=None, mode=GradientMode.Overwrite, output=None):
        check(lib().neus_module_backward(self._h, _stream(), ctx._h, C.c_uint32(ctx.n), _p(dL_dinput), _p(dL_doutput), _p(dL_dparams),
                                         _p(x), _p(output), _p(params), C.c_int(int(mode))))
        return dL_dparams, dL_dinput

    def backward_backward_input(self, ctx, x, dL_ddLdinput, dL_doutput, params, dL_dparams=None, dL_ddLdoutput=None,
                                mode=GradientMode.Overwrite):
        if self.kind == "network":
            raise NeusError("backward_backward_input: the NerfNetwork's second order is inside backward")
        check(lib().neus_module_backward_backward_input(self._h, _stream(), ctx._h, C.c_uint32(ctx.n), _p(dL_ddLdinput), _p(x),
                                                        _p(dL_doutput), _p(dL_dparams), _p(dL_ddLdoutput), None, _p(params),
                                                        C.c_int(int(mode))))
        return dL_dparams, dL_ddLdoutput


def create_network(n_input_dims, n_output_dims, network, batch_capacity=1 << 18):
    return Module.create_network(n_input_dims, n_output_dims, network, batch_capacity)


def create_nerf_network(config, batch_capacity=1 << 18):
    return Module.create_nerf_network(config, batch_capacity)


def create_encoding(encoding, batch_capacity=1 << 18, n_input_dims=3, requested_precision=Precision.Fp16):
    return Module.create_encoding(encoding, batch_capacity, n_input_dims, requested_precision)


def create_network_with_input_encoding(n_input_dims, n_output_dims, encoding, network, batch_capacity=1 << 18):
    return Module.create_network_with_input_encoding(n_input_dims, n_output_dims, encoding, network, batch_capacity)
