// drop_in.cpp — a C++ caller of the engine written the way the reference's Testbed calls tiny-cuda-nn
// (include/ngp_tcnn_adapter.hpp over include/ngp_engine.h). Built with g++ alone (no HIP/CUDA headers):
// the boundary is plain C. tests/test_gpu_dropin.py runs it on the GPU and checks its outputs against
// the CPU oracle.
//
// usage: drop_in <dir> <n>
//   reads  <dir>/{encoding,dir_encoding,network,rgb_network,optimizer}.json, coords.bin (f32 [n x 7],
//          NerfCoordinate), dL.bin (f16 [n x 16])
//   writes <dir>/params.bin (f16 [n_params], after initialisation), infer.bin (f16 [n x 16] CM),
//          density.bin (f16 [16 x n] RM), fwd.bin (f16 [n x 16]), grads.bin (f16 [n_params]),
//          params_after.bin (f16 [n_params] after optimizer_step(128)), meta.json; then, on the restored
//          parameters: normals.bin (f32 [n x 7]: input_gradient(dim 3) written over a copy of the
//          coordinates, as testbed_nerf.cu:2616 does), dinput.bin (f32 [n x 7]: backward's dL_dinput),
//          dens_out.bin (f16 [n x 16]: density_forward), grads2.bin (f16 [n_params] after backward +
//          density_backward with dL.bin as dL/d(density output)), dens_dinput.bin (f32 [n x 7])
// The Testbed's sequence per step (testbed_nerf.cu:3514, 4001, 4077-4078, 3678): density for the
// occupancy grid, inference over the samples, forward + backward on the batch, optimizer_step.
#include <cstdio>
#include <fstream>
#include <iterator>
#include <sstream>
#include <string>
#include <vector>

#include "ngp_tcnn_adapter.hpp"

using namespace ngp_mi355x;

static std::string slurp(const std::string& path) {
	std::ifstream f(path, std::ios::binary);
	if (!f) throw std::runtime_error("cannot open " + path);
	return std::string(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
}
static void dump(const std::string& path, const void* host, size_t bytes) {
	std::ofstream f(path, std::ios::binary);
	f.write((const char*)host, (std::streamsize)bytes);
}

// device buffer owned through the C-ABI's allocator (the reference would use tcnn::GPUMemory)
struct DevBuf {
	void* p = nullptr;
	size_t bytes = 0;
	explicit DevBuf(size_t b) : bytes(b) { check(ngp_malloc(&p, b), "ngp_malloc"); }
	~DevBuf() { ngp_free(p); }
	void upload(const void* host) { check(ngp_memcpy(p, host, bytes, 1 /* hipMemcpyHostToDevice */), "upload"); }
	void download(void* host, size_t b) const { check(ngp_memcpy(host, p, b, 2 /* hipMemcpyDeviceToHost */), "download"); }
};

int main(int argc, char** argv) {
	if (argc != 3) {
		fprintf(stderr, "usage: %s <dir> <n>\n", argv[0]);
		return 2;
	}
	const std::string dir = argv[1];
	const uint32_t n = (uint32_t)std::stoul(argv[2]);
	try {
		NerfNetwork net(3, 3, 0, 4, slurp(dir + "/encoding.json"), slurp(dir + "/dir_encoding.json"), slurp(dir + "/network.json"),
		                slurp(dir + "/rgb_network.json"));
		Trainer trainer(net, slurp(dir + "/optimizer.json"), 1337);
		const uint64_t np = net.n_params();
		const uint32_t W = net.padded_output_width();

		const std::string coords = slurp(dir + "/coords.bin"), dl = slurp(dir + "/dL.bin");
		if (coords.size() != (size_t)n * 7 * 4 || dl.size() != (size_t)n * 16 * 2) throw std::runtime_error("input sizes");
		DevBuf d_coords(coords.size()), d_dl(dl.size()), d_out((size_t)n * W * 2), d_den((size_t)16 * n * 2), d_fwd((size_t)n * W * 2);
		d_coords.upload(coords.data());
		d_dl.upload(dl.data());
		void* stream = nullptr;  // default stream; the Testbed passes its m_stream.get()

		std::vector<uint16_t> h16(np);
		check(ngp_memcpy(h16.data(), trainer.params(), np * 2, 2), "params");
		dump(dir + "/params.bin", h16.data(), np * 2);

		const MatrixView<const float> in{(const float*)d_coords.p, 7, n, 7, Layout::CM};
		net.inference_mixed_precision(stream, in, MatrixView<uint16_t>{(uint16_t*)d_out.p, W, n, W, Layout::CM}, false);
		net.density(stream, in, MatrixView<uint16_t>{(uint16_t*)d_den.p, 16, n, n, Layout::RM}, false);
		MatrixView<uint16_t> fwd{(uint16_t*)d_fwd.p, W, n, W, Layout::CM};
		auto ctx = net.forward(stream, in, &fwd, false);
		net.backward(stream, *ctx, MatrixView<const uint16_t>{(const uint16_t*)d_dl.p, 16, n, 16, Layout::CM});
		check(ngp_stream_synchronize(stream), "sync");

		std::vector<uint16_t> o((size_t)n * W);
		d_out.download(o.data(), o.size() * 2);
		dump(dir + "/infer.bin", o.data(), o.size() * 2);
		d_den.download(o.data(), (size_t)16 * n * 2);
		dump(dir + "/density.bin", o.data(), (size_t)16 * n * 2);
		d_fwd.download(o.data(), o.size() * 2);
		dump(dir + "/fwd.bin", o.data(), o.size() * 2);
		check(ngp_memcpy(h16.data(), trainer.gradients(), np * 2, 2), "gradients");
		dump(dir + "/grads.bin", h16.data(), np * 2);

		const std::vector<uint8_t> snap = trainer.serialize();
		trainer.optimizer_step(stream, 128.0f);
		check(ngp_stream_synchronize(stream), "sync");
		check(ngp_memcpy(h16.data(), trainer.params(), np * 2, 2), "params");
		dump(dir + "/params_after.bin", h16.data(), np * 2);
		const uint32_t step_after = trainer.step();
		trainer.deserialize(snap);  // Trainer::deserialize restores the pre-step state
		const uint32_t step_restored = trainer.step();

		// normals (testbed_nerf.cu:2616): network.input_gradient(stream, 3, positions_matrix, positions_matrix)
		DevBuf d_pos(coords.size());
		d_pos.upload(coords.data());
		net.input_gradient(stream, 3, MatrixView<const float>{(const float*)d_pos.p, 7, n, 7, Layout::CM},
		                   MatrixView<float>{(float*)d_pos.p, 7, n, 7, Layout::CM});
		// backward with input gradients (nerf_network.h:262), then density_forward / density_backward (:355-428)
		const std::vector<float> zeros((size_t)n * 7, 0.f);
		DevBuf d_din(zeros.size() * 4), d_ddin(zeros.size() * 4), d_dout((size_t)n * 16 * 2);
		d_din.upload(zeros.data());
		d_ddin.upload(zeros.data());
		auto ctx2 = net.forward(stream, in, &fwd, false);
		MatrixView<float> din{(float*)d_din.p, 7, n, 7, Layout::CM}, ddin{(float*)d_ddin.p, 7, n, 7, Layout::CM};
		net.backward(stream, *ctx2, MatrixView<const uint16_t>{(const uint16_t*)d_dl.p, 16, n, 16, Layout::CM}, &din);
		MatrixView<uint16_t> dout{(uint16_t*)d_dout.p, 16, n, 16, Layout::CM};
		auto dctx = net.density_forward(stream, in, &dout, false);
		net.density_backward(stream, *dctx, MatrixView<const uint16_t>{(const uint16_t*)d_dl.p, 16, n, 16, Layout::CM}, &ddin);
		check(ngp_stream_synchronize(stream), "sync");
		std::vector<float> f32v(zeros.size());
		d_pos.download(f32v.data(), f32v.size() * 4);
		dump(dir + "/normals.bin", f32v.data(), f32v.size() * 4);
		d_din.download(f32v.data(), f32v.size() * 4);
		dump(dir + "/dinput.bin", f32v.data(), f32v.size() * 4);
		d_ddin.download(f32v.data(), f32v.size() * 4);
		dump(dir + "/dens_dinput.bin", f32v.data(), f32v.size() * 4);
		d_dout.download(o.data(), (size_t)n * 16 * 2);
		dump(dir + "/dens_out.bin", o.data(), (size_t)n * 16 * 2);
		check(ngp_memcpy(h16.data(), trainer.gradients(), np * 2, 2), "gradients");
		dump(dir + "/grads2.bin", h16.data(), np * 2);
		std::string ctx_err;  // a forward() context handed to density_backward is refused
		try {
			auto ctx3 = net.forward(stream, in, &fwd, false);
			net.density_backward(stream, *ctx3, MatrixView<const uint16_t>{(const uint16_t*)d_dl.p, 16, n, 16, Layout::CM});
		} catch (const std::runtime_error& e) {
			ctx_err = e.what();
		}

		// the reference's error behaviour: a non-CM input throws (nerf_network.h:338-340)
		std::string err;
		try {
			net.density(stream, MatrixView<const float>{(const float*)d_coords.p, 7, n, n, Layout::RM},
			            MatrixView<uint16_t>{(uint16_t*)d_den.p, 16, n, n, Layout::RM});
		} catch (const std::runtime_error& e) {
			err = e.what();
		}
		std::ostringstream meta;
		meta << "{\"n_params\": " << np << ", \"n_matrix_params\": " << net.n_matrix_params() << ", \"padded_output_width\": " << W
		     << ", \"input_width\": " << net.input_width() << ", \"output_width\": " << net.output_width()
		     << ", \"step_after\": " << step_after << ", \"step_restored\": " << step_restored
		     << ", \"learning_rate\": " << trainer.learning_rate() << ", \"serialized_bytes\": " << snap.size()
		     << ", \"rm_input_error\": \"" << err << "\", \"ctx_kind_error\": \"" << (ctx_err.empty() ? "" : "refused") << "\"}";
		std::ofstream(dir + "/meta.json") << meta.str();
	} catch (const std::exception& e) {
		fprintf(stderr, "drop_in: %s\n", e.what());
		return 1;
	}
	return 0;
}
