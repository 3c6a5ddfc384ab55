"""Host-side mirror of the reference's model/trainer interface over the C-ABI.

Names and argument meaning follow the objects the reference's Testbed drives
(tcnn::NetworkWithInputEncoding, ngp::NerfNetwork — include/neural-graphics-primitives/nerf_network.h,
tcnn::Trainer — src/testbed.cu:4129). Device buffers are torch tensors (PyTorch is plumbing for
device memory, streams and torch.distributed here); every compute call goes to the HIP engine.
"""
import ctypes as C
import json

import torch

from ._capi import NgpError, ParamLayout, check, lib

LAYOUT_AOS, LAYOUT_SOA = 0, 1
LAYOUT_AOS_RGBD = 2  # engine extension: NerfNetwork rows 0..3 only (raw rgb, raw density), [n x 4]
GRAD_OVERWRITE, GRAD_ACCUMULATE, GRAD_IGNORE = 0, 1, 2  # tcnn::EGradientMode


def _js(cfg):
    if cfg is None:
        return None
    return (cfg if isinstance(cfg, str) else json.dumps(cfg)).encode()


def _stream(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _check_input(x, width):
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.stride(1) == 1):
        raise ValueError("input must be a CUDA float32 [n, stride] row-major tensor")
    if x.shape[1] < width:
        raise ValueError(f"input has {x.shape[1]} columns, the model reads {width}")


class _CudaArray:
    """Exposes an engine-owned device buffer to torch via __cuda_array_interface__."""

    def __init__(self, ptr, n, typestr):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False), "version": 3, "strides": None}


def wrap_device(ptr, n, dtype):
    typestr = {torch.float16: "<f2", torch.float32: "<f4"}[dtype]
    return torch.as_tensor(_CudaArray(ptr, n, typestr), device="cuda")


def _destroy(obj, fn):
    h = getattr(obj, "handle", None)
    if h:
        try:
            getattr(lib(), fn)(h)
        except Exception:  # interpreter teardown: module globals may already be gone
            pass
        obj.handle = None


class Context:
    def __init__(self, model, handle, n):
        self.model, self.handle, self.n = model, handle, n

    def __del__(self, _d=_destroy):
        _d(self, "ngp_ctx_destroy")


class Model:
    """Common surface of tcnn::Network<float, __half> as the Testbed uses it."""

    def __init__(self, handle):
        self.handle = handle
        self._keep = []

    def __del__(self, _d=_destroy):
        _d(self, "ngp_model_destroy")

    # -- shape queries ------------------------------------------------------------------------
    @property
    def n_params(self):
        return lib().ngp_model_n_params(self.handle)

    @property
    def n_matrix_params(self):
        return lib().ngp_model_n_matrix_params(self.handle)

    def input_width(self):
        return lib().ngp_model_input_width(self.handle)

    def padded_output_width(self):
        return lib().ngp_model_padded_output_width(self.handle)

    def output_width(self):
        return lib().ngp_model_output_width(self.handle)

    def layout(self):
        lo = ParamLayout()
        check(lib().ngp_model_param_layout(self.handle, C.byref(lo)))
        return lo

    # -- parameters ---------------------------------------------------------------------------
    def set_params(self, params, inference_params=None, gradients=None):
        for t in (params, inference_params, gradients):
            if t is not None and (t.dtype != torch.float16 or t.numel() != self.n_params or not t.is_cuda):
                raise ValueError("parameter buffers must be CUDA fp16 tensors of n_params elements")
        self._keep = [params, inference_params, gradients]
        check(lib().ngp_model_set_params(self.handle, _ptr(params), _ptr(inference_params), _ptr(gradients)))

    def initialize_params(self, seed=1337, scale=1.0):
        import numpy as np
        out = np.zeros(self.n_params, dtype=np.float32)
        check(lib().ngp_model_initialize_params(self.handle, seed, out.ctypes.data_as(C.c_void_p), scale))
        return out

    def set_max_level(self, max_level=1.0, per_sample=None):
        self._max_level_keep = per_sample
        check(lib().ngp_model_set_max_level(self.handle, float(max_level), _ptr(per_sample)))

    def set_option(self, key, value):
        check(lib().ngp_model_set_option(self.handle, key.encode(), float(value)))

    def query(self, key):
        """engine state (ngp_model_query): "grid_brick_levels" """
        v = C.c_double()
        check(lib().ngp_model_query(self.handle, key.encode(), C.byref(v)))
        return v.value

    def reserve(self, n):
        check(lib().ngp_model_reserve(self.handle, n))

    def workspace(self, name, n):
        """The last training pass's fp16 intermediates as a [n x width] view: "encoding" (grid output) or
        "dL_dencoding" (grid backward input), width encoding_width — tcnn's forward_activations(ctx) role —
        or "dL_dsh" (dL/d(SH encoding) of the last backward with input gradients), width 16."""
        p, nb = C.c_void_p(), C.c_uint64()
        check(lib().ngp_model_workspace(self.handle, name.encode(), C.byref(p), C.byref(nb)))
        w = 16 if name == "dL_dsh" else self.layout().encoding_width
        if n * w * 2 > nb.value:
            raise ValueError(f"workspace {name} holds {nb.value} bytes, fewer than {n} rows")
        return wrap_device(p.value, n * w, torch.float16).view(n, w)

    # -- compute ------------------------------------------------------------------------------
    def inference(self, x, output=None, layout=LAYOUT_AOS, use_inference_params=True, stream=None):
        _check_input(x, self.input_width())
        n = x.shape[0]
        if output is None:
            shape = {LAYOUT_AOS: (n, 16), LAYOUT_SOA: (16, n), LAYOUT_AOS_RGBD: (n, 4)}[layout]
            output = torch.empty(shape, dtype=torch.float16, device=x.device)
        stride = output.stride(0)
        check(lib().ngp_inference(self.handle, _stream(stream), n, _ptr(x), x.stride(0), _ptr(output), stride, layout,
                                  int(use_inference_params)))
        return output

    def forward(self, x, output=None, use_inference_params=False, stream=None):
        _check_input(x, self.input_width())
        h = C.c_void_p()
        check(lib().ngp_forward(self.handle, _stream(stream), x.shape[0], _ptr(x), x.stride(0), _ptr(output),
                                output.stride(0) if output is not None else 0, int(use_inference_params), C.byref(h)))
        return Context(self, h, x.shape[0]), output

    def backward(self, ctx, dL_doutput, dL_dinput=None, grad_mode=GRAD_OVERWRITE, stream=None):
        """backward_impl (nerf_network.h:256-335). dL_dinput: optional fp32 [n x >= input_width] tensor that
        receives dL/dposition (and dL/ddirection for a NerfNetwork); other columns are not written."""
        assert dL_doutput.dtype == torch.float16 and dL_doutput.shape[1] >= 16
        if dL_dinput is not None:
            assert dL_dinput.dtype == torch.float32 and dL_dinput.shape[0] == ctx.n
        check(lib().ngp_backward(self.handle, _stream(stream), ctx.handle, _ptr(dL_doutput), dL_doutput.stride(0),
                                 _ptr(dL_dinput), dL_dinput.stride(0) if dL_dinput is not None else 0, grad_mode))

    def input_gradient(self, dim, x, d_dinput=None, backprop_scale=128.0, stream=None):
        """tcnn Network::input_gradient (the reference's normals: testbed_nerf.cu:2616, testbed.cu:4621):
        d output[dim] / d input, fp32 [n x input width] (only the position / direction columns written)."""
        _check_input(x, self.input_width())
        if d_dinput is None:
            d_dinput = torch.zeros((x.shape[0], x.shape[1]), dtype=torch.float32, device=x.device)
        check(lib().ngp_input_gradient(self.handle, _stream(stream), dim, x.shape[0], _ptr(x), x.stride(0), _ptr(d_dinput),
                                       d_dinput.stride(0), float(backprop_scale)))
        return d_dinput

    def forward_backward(self, x, dL_doutput, output=None, grad_mode=GRAD_OVERWRITE, stream=None):
        _check_input(x, self.input_width())
        assert dL_doutput.dtype == torch.float16 and dL_doutput.shape[1] >= 16
        check(lib().ngp_forward_backward(self.handle, _stream(stream), x.shape[0], _ptr(x), x.stride(0), _ptr(output),
                                         output.stride(0) if output is not None else 0, _ptr(dL_doutput),
                                         dL_doutput.stride(0), grad_mode))
        return output

    def encode(self, x, layout=LAYOUT_AOS, use_inference_params=False, stream=None):
        n = x.shape[0]
        w = self.layout().encoding_width
        out = torch.zeros((n, w) if layout == LAYOUT_AOS else (w, n), dtype=torch.float16, device=x.device)
        check(lib().ngp_encoding_forward(self.handle, _stream(stream), n, _ptr(x), x.stride(0), _ptr(out), out.stride(0),
                                         layout, int(use_inference_params)))
        return out

    def encoding_backward(self, x, dL_dy, layout=LAYOUT_AOS, grad_mode=GRAD_OVERWRITE, dL_dinput=None, stream=None):
        check(lib().ngp_encoding_backward(self.handle, _stream(stream), x.shape[0], _ptr(x), x.stride(0), _ptr(dL_dy),
                                          dL_dy.stride(0), layout, _ptr(dL_dinput),
                                          dL_dinput.stride(0) if dL_dinput is not None else 0, grad_mode))


class NerfNetwork(Model):
    """ngp::NerfNetwork<__half>(n_pos_dims, n_dir_dims, n_extra_dims, dir_offset, pos_encoding,
    dir_encoding, density_network, rgb_network) — nerf_network.h:81-112."""

    def __init__(self, n_pos_dims, n_dir_dims, n_extra_dims, dir_offset, pos_encoding, dir_encoding, density_network,
                 rgb_network):
        h = C.c_void_p()
        check(lib().ngp_nerf_network_create(n_pos_dims, n_dir_dims, n_extra_dims, dir_offset, _js(pos_encoding),
                                            _js(dir_encoding), _js(density_network), _js(rgb_network), C.byref(h)))
        super().__init__(h)

    def density(self, x, output=None, layout=LAYOUT_AOS, use_inference_params=True, stream=None):
        n = x.shape[0]
        if output is None:
            shape = {LAYOUT_AOS: (n, 16), LAYOUT_SOA: (16, n), LAYOUT_AOS_RGBD: (n, 4)}[layout]
            output = torch.empty(shape, dtype=torch.float16, device=x.device)
        check(lib().ngp_density(self.handle, _stream(stream), n, _ptr(x), x.stride(0), _ptr(output), output.stride(0), layout,
                                int(use_inference_params)))
        return output

    def density_forward(self, x, output=None, use_inference_params=False, stream=None):
        """NerfNetwork::density_forward (nerf_network.h:355-382): (context, density network output [n x 16])."""
        h = C.c_void_p()
        check(lib().ngp_density_forward(self.handle, _stream(stream), x.shape[0], _ptr(x), x.stride(0), _ptr(output),
                                        output.stride(0) if output is not None else 0, int(use_inference_params), C.byref(h)))
        return Context(self, h, x.shape[0]), output

    def density_backward(self, ctx, dL_doutput, dL_dinput=None, grad_mode=GRAD_OVERWRITE, stream=None):
        """NerfNetwork::density_backward (nerf_network.h:384-428): dL_doutput = dL/d(density output) fp16 [n x 16]."""
        assert dL_doutput.dtype == torch.float16 and dL_doutput.shape[1] >= 16
        check(lib().ngp_density_backward(self.handle, _stream(stream), ctx.handle, _ptr(dL_doutput), dL_doutput.stride(0),
                                         _ptr(dL_dinput), dL_dinput.stride(0) if dL_dinput is not None else 0, grad_mode))


class NetworkWithInputEncoding(Model):
    """tcnn::NetworkWithInputEncoding(n_input_dims, n_output_dims, encoding, network) — src/testbed.cu:4110."""

    def __init__(self, n_input_dims, n_output_dims, encoding, network):
        h = C.c_void_p()
        check(lib().ngp_network_with_input_encoding_create(n_input_dims, n_output_dims, _js(encoding), _js(network),
                                                           C.byref(h)))
        super().__init__(h)


LOSSES = {"L2": 0, "L1": 1, "MAPE": 2, "SMAPE": 3, "RelativeL2": 4}  # NGP_LOSS_* (tcnn loss otypes)


def loss_evaluate(loss, output, target, dims, loss_scale=128.0, stream=None):
    """tcnn Loss::evaluate restated: output fp16 [n, 16], target float32 [n, >= dims] ->
    (dL/doutput fp16 [n, 16], per-sample values float32 [n], total float)."""
    n = output.shape[0]
    dl = torch.empty((n, output.shape[1]), dtype=torch.float16, device=output.device)
    vals = torch.empty(n, dtype=torch.float32, device=output.device)
    tot = torch.zeros(1, dtype=torch.float32, device=output.device)
    check(lib().ngp_loss_evaluate(LOSSES[loss] if isinstance(loss, str) else int(loss), _stream(stream), n, dims,
                                  _ptr(output), output.stride(0), _ptr(target), target.stride(0), float(loss_scale),
                                  _ptr(dl), dl.stride(0), _ptr(vals), _ptr(tot)))
    return dl, vals, float(tot.item())


class Trainer:
    """tcnn::Trainer<float, __half, __half>(network, optimizer, loss, seed) — src/testbed.cu:4129.
    The loss is applied by the caller (NeRF computes dL/doutput itself, testbed_nerf.cu:1660-2012)."""

    def __init__(self, model, optimizer, seed=1337):
        self.model = model
        h = C.c_void_p()
        check(lib().ngp_trainer_create(model.handle, _js(optimizer), seed, C.byref(h)))
        self.handle = h
        n = model.n_params
        L = lib()
        self.gradients = wrap_device(L.ngp_trainer_gradients(h), n, torch.float16)
        self.params = wrap_device(L.ngp_trainer_params(h), n, torch.float16)

    def __del__(self, _d=_destroy):
        _d(self, "ngp_trainer_destroy")

    @property
    def params_full_precision(self):
        """The fp32 master weights. A large-table trainer keeps them in its optimizer records (optimizer.h
        AdamRec::w) and ngp_trainer_params_full_precision refreshes this mirror first; write new weights with
        set_params_full_precision (tcnn's Trainer::set_params_full_precision, testbed.cu:4146)."""
        p = lib().ngp_trainer_params_full_precision(self.handle)
        if not p:
            raise NgpError(lib().ngp_last_error().decode())
        return wrap_device(p, self.model.n_params, torch.float32)

    @property
    def inference_params(self):
        """The EMA (inference) parameters, brought up to date first: a large-table trainer keeps the EMA of
        untouched entries lazily (optimizer.h AdamRec) and ngp_trainer_inference_params completes it."""
        p = lib().ngp_trainer_inference_params(self.handle)
        if not p:
            raise NgpError(lib().ngp_last_error().decode())
        return wrap_device(p, self.model.n_params, torch.float16)

    def optimizer_step(self, loss_scale=128.0, stream=None):
        check(lib().ngp_trainer_optimizer_step(self.handle, _stream(stream), float(loss_scale)))

    @property
    def step(self):
        return lib().ngp_trainer_step(self.handle)

    @property
    def learning_rate(self):
        return lib().ngp_trainer_learning_rate(self.handle)

    @learning_rate.setter
    def learning_rate(self, lr):
        check(lib().ngp_trainer_set_learning_rate(self.handle, float(lr)))

    def set_option(self, key, value):
        """Engine trainer option (ngp_trainer_set_option), e.g. "ema_closed_form"."""
        check(lib().ngp_trainer_set_option(self.handle, key.encode(), float(value)))

    def set_params_full_precision(self, params_host):
        import numpy as np
        a = np.ascontiguousarray(params_host, dtype=np.float32)
        check(lib().ngp_trainer_set_params_full_precision(self.handle, a.ctypes.data_as(C.c_void_p), a.size))

    def training_step(self, x, target, loss="L2", loss_scale=128.0, run_optimizer=True, get_loss=True, stream=None):
        """tcnn Trainer::training_step(stream, input, target, nullptr, run_optimizer) (src/testbed_image.cu:276,
        src/testbed_sdf.cu:1304). target: CUDA float32 [n, >= output_width]. Returns the loss scalar."""
        _check_input(x, self.model.input_width())
        if not (target.is_cuda and target.dtype == torch.float32 and target.dim() == 2 and target.stride(1) == 1):
            raise ValueError("target must be a CUDA float32 [n, dims] row-major tensor")
        acc = torch.zeros(1, dtype=torch.float32, device=x.device) if get_loss else None
        check(lib().ngp_trainer_training_step(self.handle, _stream(stream), x.shape[0], _ptr(x), x.stride(0), _ptr(target),
                                              target.stride(0), LOSSES[loss] if isinstance(loss, str) else int(loss),
                                              float(loss_scale), int(run_optimizer), _ptr(acc)))
        return float(acc.item()) if get_loss else None

    def serialize(self):
        size = C.c_uint64(0)
        check(lib().ngp_trainer_serialize(self.handle, None, C.byref(size)))
        buf = C.create_string_buffer(size.value)
        check(lib().ngp_trainer_serialize(self.handle, buf, C.byref(size)))
        return buf.raw

    def deserialize(self, blob):
        check(lib().ngp_trainer_deserialize(self.handle, blob, len(blob)))

    def set_allreduce(self, comm):
        """Engine extension: all-reduce (sum) the gradient buffer with `comm` (dp.EngineComm) inside every
        captured training step, before the optimizer, which then uses the mean gradient. None: off."""
        if comm is None:
            check(lib().ngp_trainer_set_allreduce(self.handle, 1, None, None))
        else:
            check(lib().ngp_trainer_set_allreduce(self.handle, comm.world, comm.fn, comm.handle))
        self._comm = comm

    def set_data_parallel(self, comm):
        """Engine extension: the exchange of set_allreduce with this rank (comm.rank), so that large-table trainers
        shard the optimizer (reduce-scatter of the fp32-widened gradients, this rank's slice of the update,
        all-gather of the fp16 weights; option shard_opt). None: off. With world > 1, call gather_shards() on every
        rank before reading inference_params / params_full_precision or serializing."""
        if comm is None:
            check(lib().ngp_trainer_set_data_parallel(self.handle, 0, 1, None, None))
        else:
            check(lib().ngp_trainer_set_data_parallel(self.handle, comm.rank, comm.world, comm.fn, comm.handle))
        self._comm = comm

    def gather_shards(self, stream=None):
        """Collective: every rank gets the whole (sharded) optimizer state again (ngp_trainer_gather_shards)."""
        check(lib().ngp_trainer_gather_shards(self.handle, _stream(stream)))

    def train_step(self, x, dL_doutput, loss_scale=128.0, stream=None):
        """Engine extension: one eager step of what capture_training_step records (forward_backward with the
        grid's update fused into the backward where possible, the exchange hook, optimizer_step)."""
        _check_input(x, self.model.input_width())
        check(lib().ngp_trainer_train_step(self.handle, _stream(stream), x.shape[0], _ptr(x), x.stride(0),
                                           _ptr(dL_doutput), dL_doutput.stride(0), float(loss_scale)))

    def fused_update_active(self, n_batch):
        """True when a training step of n_batch samples updates the grid inside the backward (the grid part
        of the gradient buffer is then not written)."""
        return bool(lib().ngp_trainer_fused_update_active(self.handle, int(n_batch)))

    @property
    def gradients_valid(self):
        """False when the last step did not write `gradients` (the fused grid update or the sharded
        data-parallel step took the gradient without storing it as fp16): the buffer is an older one."""
        return bool(lib().ngp_trainer_gradients_valid(self.handle))

    def capture_training_step(self, x, dL_doutput, loss_scale=128.0, n_steps=1, with_optimizer=True, stream=None):
        """Engine extension: n_steps of forward_backward(x, dL_doutput) [+ optimizer_step] captured into
        one HIP graph (TrainingGraph.launch replays it). `stream` must not be the null stream."""
        s = _stream(stream)
        if not s.value:
            raise ValueError("graph capture needs a non-default stream (use torch.cuda.Stream())")
        _check_input(x, self.model.input_width())
        h = C.c_void_p()
        check(lib().ngp_trainer_capture_training_step(self.handle, s, x.shape[0], _ptr(x), x.stride(0), _ptr(dL_doutput),
                                                      dL_doutput.stride(0), float(loss_scale), n_steps, int(with_optimizer),
                                                      C.byref(h)))
        return TrainingGraph(h, (x, dL_doutput))


class TrainingGraph:
    def __init__(self, handle, keep):
        self.handle, self._keep = handle, keep

    def launch(self, stream=None):
        check(lib().ngp_graph_launch(self.handle, _stream(stream)))

    def __del__(self, _d=_destroy):
        _d(self, "ngp_graph_destroy")
