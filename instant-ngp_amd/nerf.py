"""Host mirror of the Testbed's NeRF training path (src/testbed_nerf.cu) over the C-ABI.

`NerfTraining` is Testbed::train for a NeRF testbed (training_prep_nerf + train_nerf,
testbed_nerf.cu:3611-3862, 4137-4152); the free functions expose the individual kernels
(generate_training_samples_nerf, compute_loss_kernel_train_nerf, the density-grid update) with
the reference's argument meaning so they can be tested one by one. Every call runs HIP.
"""
import ctypes as C
import json
import math
import os

import numpy as np
import torch

from ._capi import NerfConfig, NerfErrorMapInfo, NerfImage, NerfStats, Rng, check, lib
from .network import _ptr, _stream, wrap_device

NERF_GRIDSIZE = 128
NERF_CASCADES = 8
N_CELLS = NERF_GRIDSIZE ** 3
BITFIELD_BYTES = N_CELLS // 8 * NERF_CASCADES
ACT = {"None": 0, "ReLU": 1, "Logistic": 2, "Exponential": 3}
LOSS = {"L2": 0, "L1": 1, "MAPE": 2, "SMAPE": 3, "Huber": 4, "LogL1": 5, "RelativeL2": 6}


def default_config(aabb_scale=1.0, **overrides):
    """Testbed NeRF defaults after load_nerf_post (testbed_nerf.cu:3093-3109, testbed.h:716-785)."""
    cfg = NerfConfig()
    check(lib().ngp_nerf_default_config(float(aabb_scale), C.byref(cfg)))
    for k, v in overrides.items():
        if isinstance(getattr(cfg, k), C.Array):
            getattr(cfg, k)[:] = list(v)
        else:
            setattr(cfg, k, v)
    return cfg


def rng_state(state, inc):
    return Rng(state, inc)


def pcg32(seed, seq=1):
    """tcnn::pcg32(initstate, initseq) seeding (pcg32.h), host side."""
    mask = (1 << 64) - 1
    mult = 0x5851F42D4C957F2D
    inc = ((seq << 1) | 1) & mask
    state = 0
    state = (state * mult + inc) & mask
    state = (state + seed) & mask
    state = (state * mult + inc) & mask
    return Rng(state, inc)


def nerf_matrix_to_ngp(m, scale=0.33, offset=(0.5, 0.5, 0.5)):
    """NerfDataset::nerf_matrix_to_ngp (nerf_loader.h:120-140), non-mitsuba branch.
    m: 3x4 (or 4x4) camera-to-world in the NeRF/Blender convention. Returns the 12 floats of the
    column-major mat4x3 the engine takes."""
    m = np.asarray(m, dtype=np.float32)[:3, :4].copy()
    m[:, 1] *= -1.0
    m[:, 2] *= -1.0
    m[:, 3] = m[:, 3] * np.float32(scale) + np.asarray(offset, np.float32)
    m = m[[1, 2, 0], :]  # cycle axes xyz <- yzx
    return np.ascontiguousarray(m.T).reshape(12)


LENS_PERSPECTIVE, LENS_OPENCV, LENS_OPENCV_FISHEYE = 0, 1, 2


def make_image(width, height, xform12, focal=None, camera_angle_x=None, principal=(0.5, 0.5), lens_mode=LENS_PERSPECTIVE,
               lens_params=(0.0, 0.0, 0.0, 0.0)):
    im = NerfImage()
    im.width, im.height = width, height
    if focal is None:
        f = 0.5 * width / math.tan(0.5 * camera_angle_x)  # nerf_loader.cu: fl from camera_angle_x
        focal = (f, f)
    im.focal_length[:] = list(focal)
    im.principal_point[:] = list(principal)
    im.xform[:] = [float(v) for v in xform12]
    im.lens_mode = int(lens_mode)
    im.lens_params[:] = [float(v) for v in lens_params]
    return im


class NerfDataset:
    """Training images (RGBA8 sRGB, EImageDataType::Byte) + cameras on the device."""

    def __init__(self, images, rgba8):
        if len(images) != len(rgba8) or not images:
            raise ValueError("need one RGBA8 array per image")
        arr = (NerfImage * len(images))(*images)
        self.images = list(images)
        bufs = []
        for im, px in zip(images, rgba8):
            px = np.ascontiguousarray(px, dtype=np.uint8)
            if px.shape != (im.height, im.width, 4):
                raise ValueError(f"image buffer shape {px.shape} != {(im.height, im.width, 4)}")
            bufs.append(px)
        self._host = bufs
        ptrs = (C.c_void_p * len(bufs))(*[b.ctypes.data for b in bufs])
        h = C.c_void_p()
        check(lib().ngp_nerf_dataset_create(len(images), arr, ptrs, C.byref(h)))
        self.handle = h

    def __len__(self):
        return len(self.images)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                lib().ngp_nerf_dataset_destroy(h)
            except Exception:
                pass
            self.handle = None


# ---- kernel-level entry points ------------------------------------------------------------------
def generate_training_samples(ds, cfg, n_rays, rng, max_samples, bitfield, ray_offset=0, n_rays_total=None,
                              stream=None):
    """generate_training_samples_nerf (testbed_nerf.cu:1382-1658)."""
    dev = bitfield.device
    out = {
        "ray_indices": torch.zeros(n_rays, dtype=torch.int32, device=dev),
        "rays": torch.zeros((n_rays, 6), dtype=torch.float32, device=dev),
        "numsteps": torch.zeros((n_rays, 2), dtype=torch.int32, device=dev),
        "coords": torch.zeros((max_samples, 7), dtype=torch.float32, device=dev),
        "counters": torch.zeros(2, dtype=torch.int32, device=dev),
    }
    check(lib().ngp_nerf_generate_training_samples(
        ds.handle, C.byref(cfg), _stream(stream), n_rays, ray_offset, n_rays_total or n_rays, rng, max_samples,
        _ptr(bitfield), _ptr(out["ray_indices"]), _ptr(out["rays"]), _ptr(out["numsteps"]), _ptr(out["coords"]),
        _ptr(out["counters"])))
    return out


def compute_loss(ds, cfg, n_rays, rng, max_compacted, samples, network_output, mean_density, loss_scale=128.0,
                 n_rays_total=None, stream=None, error_map=None, keep_state=False, state_capacity=None):
    """compute_loss_kernel_train_nerf (testbed_nerf.cu:1660-2012). `samples` is the dict returned by
    generate_training_samples (its numsteps is rewritten to the compacted {n, base}). error_map: a
    float32 device tensor [n_images, h, w] the compacted rays' losses are added into (:1869-1899).
    keep_state: pass 1 keeps each composited sample's state for pass 2 (ngp_nerf_compute_loss_state, the
    training step's form; same outputs bit for bit). state_capacity: samples the kept state holds (default: every
    sample slot); rays reaching past it are composited again by pass 2, with the same result."""
    dev = network_output.device
    # the kernel reads one output row per sample; samples never exceed the sampler's coords buffer
    if network_output.shape[0] < samples["coords"].shape[0]:
        raise ValueError(f"network_output has {network_output.shape[0]} rows, fewer than the {samples['coords'].shape[0]} "
                         "sample slots of generate_training_samples")
    out = {
        "coords_compacted": torch.zeros((max_compacted, 7), dtype=torch.float32, device=dev),
        "dloss_doutput": torch.zeros((max_compacted, 16), dtype=torch.float16, device=dev),
        "loss": torch.zeros(n_rays, dtype=torch.float32, device=dev),
        "compacted_counter": torch.zeros(1, dtype=torch.int32, device=dev),
    }
    args = (ds.handle, C.byref(cfg), _stream(stream), n_rays, n_rays_total or n_rays, rng, max_compacted,
            _ptr(samples["counters"]), _ptr(network_output), _ptr(samples["ray_indices"]), _ptr(samples["rays"]),
            _ptr(samples["numsteps"]), _ptr(samples["coords"]), _ptr(out["coords_compacted"]), _ptr(out["dloss_doutput"]),
            _ptr(out["loss"]), _ptr(out["compacted_counter"]), _ptr(mean_density), float(loss_scale))
    if keep_state:
        if error_map is not None:
            raise ValueError("keep_state: without error_map (the C-ABI form has no error-map argument)")
        cap = samples["coords"].shape[0] if state_capacity is None else int(state_capacity)
        state = torch.empty((5, cap), dtype=torch.float32, device=dev)
        check(lib().ngp_nerf_compute_loss_state(*args, _ptr(state), cap))
    elif error_map is None:
        check(lib().ngp_nerf_compute_loss(*args))
    else:
        if error_map.dtype != torch.float32 or error_map.dim() != 3 or not error_map.is_contiguous():
            raise ValueError("error_map: a contiguous float32 tensor [n_images, h, w]")
        check(lib().ngp_nerf_compute_loss_error_map(*args, _ptr(error_map), error_map.shape[2], error_map.shape[1]))
    return out


def fill_rollover(data, n_input, rescale=False, stream=None):
    """tcnn fill_rollover / fill_rollover_and_rescale over the rows of a 2D tensor (testbed_nerf.cu:4061-4069)."""
    dtype = {torch.float32: 0, torch.float16: 1}[data.dtype]
    check(lib().ngp_nerf_fill_rollover(_stream(stream), data.shape[0], data.shape[1], _ptr(n_input), _ptr(data), dtype,
                                       int(rescale)))


def grid_generate_samples(cfg, n, rng, step, grid, n_cascades, thresh, stream=None):
    """generate_grid_samples_nerf_nonuniform (testbed_nerf.cu:635-676)."""
    pos = torch.zeros((n, 3), dtype=torch.float32, device=grid.device)
    idx = torch.zeros(n, dtype=torch.int32, device=grid.device)
    check(lib().ngp_nerf_grid_generate_samples(_stream(stream), C.byref(cfg), n, rng, step, _ptr(grid), n_cascades,
                                               float(thresh), _ptr(pos), _ptr(idx)))
    return pos, idx


def grid_splat_max(indices, density_out, density_activation, grid_tmp, stream=None, binned=False):
    """splat_grid_samples_nerf_max_nearest_neighbor (testbed_nerf.cu:678-702). density_out: the density
    network's fp16 output, row-major [16 x n] (feature-major), density in row 0. binned: the memset of grid_tmp
    and the splat in one call (ngp_nerf_grid_splat_max_cells, a counting sort by cell bin): grid_tmp is
    overwritten, every cell of it."""
    if binned:
        check(lib().ngp_nerf_grid_splat_max_cells(_stream(stream), indices.shape[0], _ptr(indices), _ptr(density_out),
                                                  density_activation, _ptr(grid_tmp), grid_tmp.numel()))
        return
    check(lib().ngp_nerf_grid_splat_max(_stream(stream), indices.shape[0], _ptr(indices), _ptr(density_out),
                                        density_activation, _ptr(grid_tmp)))


def grid_ema(decay, grid, grid_tmp, stream=None):
    """ema_grid_samples_nerf (testbed_nerf.cu:731-754)."""
    check(lib().ngp_nerf_grid_ema(_stream(stream), grid.numel(), float(decay), _ptr(grid), _ptr(grid_tmp)))


def grid_mean_and_bitfield(grid, max_cascade, stream=None):
    """update_density_grid_mean_and_bitfield (testbed_nerf.cu:3538-3567)."""
    mean = torch.zeros(1 + 512, dtype=torch.float32, device=grid.device)
    bf = torch.zeros(BITFIELD_BYTES, dtype=torch.uint8, device=grid.device)
    check(lib().ngp_nerf_grid_mean_and_bitfield(_stream(stream), _ptr(grid), max_cascade, _ptr(mean), _ptr(bf)))
    return mean, bf


# ---- Testbed-level training -------------------------------------------------------------------
class NerfTraining:
    """Testbed::train for NeRF: density-grid update + one training step per call (testbed.cu:4285-4370)."""

    def __init__(self, network, trainer, dataset, cfg=None, seed=1337):
        self.network, self.trainer, self.dataset = network, trainer, dataset
        self.cfg = cfg if cfg is not None else default_config()
        h = C.c_void_p()
        check(lib().ngp_nerf_trainer_create(network.handle, trainer.handle, dataset.handle, C.byref(self.cfg), seed,
                                            C.byref(h)))
        self.handle = h

    def _buffers(self, write=False):
        # reads keep a prelaunched (pipelined) sampler: it reads only the bitfield and writes none of the
        # three buffers. ngp_nerf_trainer_buffers (write=True) discards it, so writes through the returned
        # views are seen by the next step's sampling
        g, b, m = C.c_void_p(), C.c_void_p(), C.c_void_p()
        fn = lib().ngp_nerf_trainer_buffers if write else lib().ngp_nerf_trainer_buffers_read
        check(fn(self.handle, C.byref(g), C.byref(b), C.byref(m)))
        return g.value, b.value, m.value

    def _views(self, write):
        g, b, m = self._buffers(write)
        return (wrap_device(g, N_CELLS * (self.cfg.max_cascade + 1), torch.float32),
                wrap_device(b, BITFIELD_BYTES // 4, torch.float32).view(torch.uint8),
                wrap_device(m, 1, torch.float32))

    @property
    def density_grid(self):
        """fp32 [128^3 x (max_cascade + 1)] (testbed_nerf.cu:3412-3420), Morton order per cascade. For
        reading (logging, snapshots); modify through writable_buffers()."""
        return self._views(False)[0]

    @property
    def mean_density(self):
        return self._views(False)[2]

    @property
    def bitfield(self):
        return self._views(False)[1]

    def writable_buffers(self):
        """(density_grid, bitfield, mean_density) views for MODIFYING the occupancy state between steps:
        discards a prelaunched sampler so the next step samples with the caller's writes."""
        return self._views(True)

    def set_data_parallel(self, rank, world, group=None, exchange_at_world_1=False):
        """Shard the rays (global ids kept), the compacted batch and the density-grid evaluation over
        `world` ranks; gradients, density-grid maxima and counters are all-reduced by the engine's RCCL
        communicator (nccl backend) or through torch.distributed (gloo: dp.make_allreduce_callback).
        exchange_at_world_1: run the data-parallel step (exchanges included) with one rank too — on a
        one-GPU box, the way to exercise the RCCL path (it must then train bitwise like the plain step)."""
        import torch.distributed as dist
        from .dp import EngineComm, make_allreduce_callback
        self._allreduce = None
        if (world > 1 or exchange_at_world_1) and dist.get_backend(group) == "nccl":
            # one GPU per rank: the engine's RCCL communicator, enqueued on the training stream
            self._allreduce = EngineComm(rank, world, group)
            fn, user = self._allreduce.fn, self._allreduce.handle
        elif world > 1:
            # gloo (CPU tests, ranks sharing a GPU): host round trip through torch.distributed
            self._allreduce = make_allreduce_callback(group)
            fn, user = C.cast(self._allreduce, C.c_void_p), None
        else:
            fn, user = None, None
        check(lib().ngp_nerf_trainer_set_data_parallel(self.handle, rank, world, fn, user))

    def set_pipeline(self, enable):
        """Launch the next step's ray sampling under this step's training pass (default on; identical
        samples). Reading density_grid / bitfield / mean_density keeps it; writable_buffers() discards it,
        so writes through those views reach the next step."""
        check(lib().ngp_nerf_trainer_set_pipeline(self.handle, int(enable)))

    def save_snapshot(self, path, network_config=None, include_optimizer_state=False, compress=True, stream=None):
        """Testbed::save_snapshot (testbed.cu:4873-4937): .ingp = gzip'd msgpack of the network config
        (dict, the Testbed's m_network_config) with the "snapshot" member."""
        cfg = json.dumps(network_config) if network_config is not None else None
        check(lib().ngp_nerf_save_snapshot(self.handle, _stream(stream), os.fsencode(path),
                                           cfg.encode() if cfg else None, int(include_optimizer_state), int(compress)))

    def load_snapshot(self, path, stream=None):
        """Testbed::load_snapshot (testbed.cu:4939-5057) into this trainer's network/optimizer/grid."""
        check(lib().ngp_nerf_load_snapshot(self.handle, _stream(stream), os.fsencode(path)))

    ERROR_MAP_ARRAYS = ("data", "cdf_x_cond_y", "cdf_y", "cdf_img", "pmf_img")

    def error_map(self):
        """The training error map (Testbed::Nerf::Training::ErrorMap, testbed.h:668-677): the rays' losses
        deposited since the current window started ("data", [n_images, h, w]) and, once a window has closed,
        its CDFs ("cdf_x_cond_y" [n_images, cdf_h, cdf_w], "cdf_y" [n_images, cdf_h], "cdf_img", "pmf_img"
        [n_images]), plus the window state (testbed_nerf.cu:3659-3666, 3700-3748)."""
        info = NerfErrorMapInfo()
        check(lib().ngp_nerf_trainer_error_map(self.handle, 0, None, 0, C.byref(info)))
        out = {k: getattr(info, k) for k, _ in NerfErrorMapInfo._fields_ if k != "size"}
        shapes = {"data": (info.n_images, info.height, info.width),
                  "cdf_x_cond_y": (info.n_images, info.cdf_height, info.cdf_width),
                  "cdf_y": (info.n_images, info.cdf_height), "cdf_img": (info.n_images,), "pmf_img": (info.n_images,)}
        for which, name in enumerate(self.ERROR_MAP_ARRAYS):
            check(lib().ngp_nerf_trainer_error_map(self.handle, which, None, 0, C.byref(info)))
            a = np.zeros(int(info.size), np.float32)
            if a.size:
                check(lib().ngp_nerf_trainer_error_map(self.handle, which, a.ctypes.data, a.size, C.byref(info)))
                a = a.reshape(shapes[name])
            out[name] = a
        return out

    def train_step(self, get_loss=True, stream=None):
        st = NerfStats()
        check(lib().ngp_nerf_train_step(self.handle, _stream(stream), int(get_loss), C.byref(st)))
        return {k: getattr(st, k) for k, _ in NerfStats._fields_}

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                lib().ngp_nerf_trainer_destroy(h)
            except Exception:
                pass
            self.handle = None


def snapshot_network_config(path):
    """Testbed::load_network_config (testbed.cu:246) of a snapshot: the network config dict without its
    "snapshot" member, e.g. to build the network before NerfTraining.load_snapshot."""
    size = C.c_uint64(0)
    check(lib().ngp_snapshot_network_config(os.fsencode(path), None, C.byref(size)))
    buf = C.create_string_buffer(size.value)
    check(lib().ngp_snapshot_network_config(os.fsencode(path), buf, C.byref(size)))
    return json.loads(buf.value.decode())


# ---- rendering / evaluation -------------------------------------------------------------------
class NerfRenderer:
    """NerfTracer (testbed_nerf.cu:2229-2659): renders a camera view with the network, marching the
    occupancy bitfield. Output: linear RGBA [H, W, 4] float32 composited over `background` (linear)."""

    def __init__(self):
        h = C.c_void_p()
        check(lib().ngp_nerf_renderer_create(C.byref(h)))
        self.handle = h

    RENDER_MODES = {"AO": 0, "Shade": 1, "Normals": 2, "Positions": 3, "Depth": 4, "EncodingVis": 9}  # ERenderMode (common.h:110-121)

    def render(self, network, cfg, camera, bitfield=None, spp=1, sample_index=0, min_transmittance=0.01,
               background=(0.0, 0.0, 0.0, 0.0), use_inference_params=True, stream=None, render_mode="Shade",
               depth_scale=1.0, show_accel=-1):
        """render_mode: an ERenderMode name; depth_scale (Depth): 1 / the dataset's scale (testbed_nerf.cu:2822);
        show_accel: Testbed::Nerf::show_accel (-1 off; 0..7: the march's minimum mip, opaque steps, Positions by cell)."""
        check(lib().ngp_nerf_renderer_set_mode(self.handle, self.RENDER_MODES[render_mode]))
        check(lib().ngp_nerf_renderer_set_show_accel(self.handle, int(show_accel)))
        check(lib().ngp_nerf_renderer_set_depth_scale(self.handle, float(depth_scale)))
        out = torch.empty((camera.height, camera.width, 4), dtype=torch.float32, device="cuda")
        bg = (C.c_float * 4)(*[float(v) for v in background])
        check(lib().ngp_nerf_render(self.handle, network.handle, C.byref(cfg), _stream(stream), C.byref(camera),
                                    _ptr(bitfield), spp, sample_index, float(min_transmittance), bg,
                                    int(use_inference_params), _ptr(out)))
        return out

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                lib().ngp_nerf_renderer_destroy(h)
            except Exception:
                pass
            self.handle = None


def linear_to_srgb(x):
    return torch.where(x < 0.0031308, 12.92 * x, 1.055 * torch.pow(torch.clamp(x, min=0), 0.41666) - 0.055)


def srgb_to_linear(x):
    return torch.where(x <= 0.04045, x / 12.92, torch.pow((x + 0.055) / 1.055, 2.4))


def ground_truth_linear(rgba8, background=(0.0, 0.0, 0.0)):
    """The reference's render_ground_truth of a training/test image (sRGB RGBA8, premultiplied by
    alpha in linear space, composited over the linear background), as a float [H, W, 4] tensor."""
    px = torch.as_tensor(rgba8).float() / 255.0
    a = px[..., 3:4]
    rgb = srgb_to_linear(px[..., :3]) * a + torch.tensor(background, dtype=torch.float32, device=px.device) * (1 - a)
    return torch.cat([rgb, torch.ones_like(a)], dim=-1)


def psnr(image, ref):
    """scripts/run.py:245-252: MSE of clip(linear_to_srgb(rgb), 0, 1), PSNR = -10 log10(MSE)."""
    A = torch.clamp(linear_to_srgb(image[..., :3].float()), 0.0, 1.0)
    R = torch.clamp(linear_to_srgb(ref[..., :3].float().to(A.device)), 0.0, 1.0)
    mse = float(torch.mean((A - R) ** 2))
    return -10.0 * math.log10(max(mse, 1e-12)), mse
