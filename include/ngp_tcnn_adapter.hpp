// ngp_tcnn_adapter.hpp — the reference-side binding: C++ classes with the tiny-cuda-nn surface the
// Testbed drives, forwarding to the C-ABI of include/ngp_engine.h. Header-only, plain C++17: it needs
// neither HIP nor CUDA headers (streams are `void*`, fp16 buffers `uint16_t*`), so a maintainer can
// include it from the reference's host code and link -lngp_engine.
//
// tcnn surface mirrored (names and argument meaning):
//   NerfNetwork<__half>                      nerf_network.h:77-578 (ctor :81-112)
//     inference_mixed_precision(stream, input, output, use_inference_params)   :116-174
//     forward(stream, input, output, use_inference_params) -> Context          :179-254
//     backward(stream, ctx, dL_doutput, dL_dinput, grad_mode)                   :256-335
//     input_gradient(stream, dim, input, d_dinput, backprop_scale)   tcnn Network; testbed_nerf.cu:2616, testbed.cu:4621
//     density(stream, input, output, use_inference_params)                      :337-353
//     density_forward / density_backward                                       :355-428
//     n_params / padded_output_width / input_width / output_width / layer_sizes :459-490
//   NetworkWithInputEncoding                 src/testbed.cu:4101-4110
//   Trainer (optimizer_step, params, serialize, set_params_full_precision)      src/testbed.cu:4129-4146,
//                                                                               testbed_nerf.cu:3678
// Errors: the reference throws std::runtime_error (CUDA_CHECK_THROW); every C-ABI failure is turned
// back into one here, carrying ngp_last_error().
#pragma once

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "ngp_engine.h"

namespace ngp_mi355x {

inline void check(int rc, const char* what) {
	if (rc != NGP_OK) throw std::runtime_error(std::string(what) + ": " + ngp_last_error());
}

// tcnn::GPUMatrixDynamic view: a device pointer plus its shape. CM (tcnn "column major") = AoS, one
// sample's features contiguous (element (i, f) at data[i * stride + f]); RM = SoA (data[f * stride + i]).
enum class Layout { CM = NGP_LAYOUT_AOS, RM = NGP_LAYOUT_SOA };
template <typename T>
struct MatrixView {
	T* data = nullptr;
	uint32_t rows = 0;     // features
	uint32_t n = 0;        // samples (tcnn: cols of a CM matrix)
	uint32_t stride = 0;   // elements between consecutive samples (CM) or features (RM)
	Layout layout = Layout::CM;
};

enum class GradientMode { Ignore = NGP_GRAD_IGNORE, Overwrite = NGP_GRAD_OVERWRITE, Accumulate = NGP_GRAD_ACCUMULATE };  // tcnn::EGradientMode

class Context {  // tcnn::Context of forward(), consumed by backward()
public:
	explicit Context(ngp_ctx* c) : c_(c) {}
	~Context() { if (c_) ngp_ctx_destroy(c_); }
	Context(const Context&) = delete;
	Context& operator=(const Context&) = delete;
	ngp_ctx* get() const { return c_; }
private:
	ngp_ctx* c_;
};

// Common tcnn::Network<float, __half> surface over an ngp_model.
class Network {
public:
	Network(const Network&) = delete;
	Network& operator=(const Network&) = delete;
	virtual ~Network() { if (m_) ngp_model_destroy(m_); }

	uint64_t n_params() const { return ngp_model_n_params(m_); }
	uint32_t input_width() const { return ngp_model_input_width(m_); }
	uint32_t padded_output_width() const { return ngp_model_padded_output_width(m_); }
	uint32_t output_width() const { return ngp_model_output_width(m_); }
	uint64_t n_matrix_params() const { return ngp_model_n_matrix_params(m_); }  // sum of layer_sizes()
	ngp_param_layout param_layout() const {
		ngp_param_layout l{};
		check(ngp_model_param_layout(m_, &l), "param_layout");
		return l;
	}
	ngp_model* handle() const { return m_; }

	// inference_mixed_precision: output fp16 [n x padded_output_width] (CM) or its transpose (RM)
	void inference_mixed_precision(void* stream, const MatrixView<const float>& input, const MatrixView<uint16_t>& output,
	                               bool use_inference_params = true) {
		require_cm(input, "inference_mixed_precision");
		check(ngp_inference(m_, stream, input.n, input.data, input.stride, output.data, output.stride,
		                    (uint32_t)output.layout, use_inference_params ? 1 : 0),
		      "inference_mixed_precision");
	}
	// forward with a context for backward(); output may be null (NerfNetwork::forward_impl, :179)
	std::unique_ptr<Context> forward(void* stream, const MatrixView<const float>& input, MatrixView<uint16_t>* output,
	                                 bool use_inference_params = false) {
		require_cm(input, "forward");
		ngp_ctx* c = nullptr;
		check(ngp_forward(m_, stream, input.n, input.data, input.stride, output ? output->data : nullptr,
		                  output ? output->stride : 0, use_inference_params ? 1 : 0, &c),
		      "forward");
		return std::unique_ptr<Context>(new Context(c));
	}
	// backward: parameter gradients into the trainer's gradient buffer (tcnn EGradientMode); dL_dinput (CM,
	// fp32) receives the input gradients when given (nerf_network.h:262, 282-299, 317-333)
	void backward(void* stream, const Context& ctx, const MatrixView<const uint16_t>& dL_doutput,
	              MatrixView<float>* dL_dinput = nullptr, GradientMode mode = GradientMode::Overwrite) {
		if (dL_dinput && dL_dinput->layout != Layout::CM) throw std::runtime_error("backward: dL_dinput must be in column major format");
		check(ngp_backward(m_, stream, ctx.get(), dL_doutput.data, dL_doutput.stride, dL_dinput ? dL_dinput->data : nullptr,
		                   dL_dinput ? dL_dinput->stride : 0, (int)mode),
		      "backward");
	}
	// tcnn Network::input_gradient: d output[dim] / d input (the reference's normals). d_dinput may be the
	// input matrix itself, as testbed_nerf.cu:2616 passes it.
	void input_gradient(void* stream, uint32_t dim, const MatrixView<const float>& input, const MatrixView<float>& d_dinput,
	                    float backprop_scale = 128.f) {
		require_cm(input, "input_gradient");
		check(ngp_input_gradient(m_, stream, dim, input.n, input.data, input.stride, d_dinput.data, d_dinput.stride, backprop_scale),
		      "input_gradient");
	}
	// GridEncoding::set_max_level / set_max_level_gpu (src/testbed.cu:3856-3864; testbed_nerf.cu:3996,4004)
	void set_max_level(float max_level, const float* max_level_per_sample_gpu = nullptr) {
		check(ngp_model_set_max_level(m_, max_level, max_level_per_sample_gpu), "set_max_level");
	}

protected:
	Network() = default;
	static void require_cm(const MatrixView<const float>& m, const char* what) {
		// the reference: "NerfNetwork::... input must be in column major format" (nerf_network.h:338-340)
		if (m.layout != Layout::CM) throw std::runtime_error(std::string(what) + ": input must be in column major format");
	}
	ngp_model* m_ = nullptr;
};

// ngp::NerfNetwork<__half>: config sections as the Testbed passes them (src/testbed.cu:4029-4042)
class NerfNetwork : public Network {
public:
	NerfNetwork(uint32_t n_pos_dims, uint32_t n_dir_dims, uint32_t n_extra_dims, uint32_t dir_offset, const std::string& encoding,
	            const std::string& dir_encoding, const std::string& density_network, const std::string& rgb_network) {
		check(ngp_nerf_network_create(n_pos_dims, n_dir_dims, n_extra_dims, dir_offset, encoding.c_str(), dir_encoding.c_str(),
		                              density_network.c_str(), rgb_network.c_str(), &m_),
		      "NerfNetwork");
	}
	// NerfNetwork::density (nerf_network.h:337-353): density MLP output, 16 rows, RM by default as the
	// density-grid update asks for it (testbed_nerf.cu:3507-3514)
	void density(void* stream, const MatrixView<const float>& input, const MatrixView<uint16_t>& output,
	             bool use_inference_params = true) {
		require_cm(input, "density");
		check(ngp_density(m_, stream, input.n, input.data, input.stride, output.data, output.stride, (uint32_t)output.layout,
		                  use_inference_params ? 1 : 0),
		      "density");
	}
	// NerfNetwork::density_forward / density_backward (nerf_network.h:355-428): the density network alone,
	// its 16-row output CM; backward writes density-MLP and grid gradients (and dL/dposition if asked)
	std::unique_ptr<Context> density_forward(void* stream, const MatrixView<const float>& input, MatrixView<uint16_t>* output,
	                                         bool use_inference_params = false) {
		require_cm(input, "density_forward");
		ngp_ctx* c = nullptr;
		check(ngp_density_forward(m_, stream, input.n, input.data, input.stride, output ? output->data : nullptr,
		                          output ? output->stride : 0, use_inference_params ? 1 : 0, &c),
		      "density_forward");
		return std::unique_ptr<Context>(new Context(c));
	}
	void density_backward(void* stream, const Context& ctx, const MatrixView<const uint16_t>& dL_doutput,
	                      MatrixView<float>* dL_dinput = nullptr, GradientMode mode = GradientMode::Overwrite) {
		if (dL_dinput && dL_dinput->layout != Layout::CM)
			throw std::runtime_error("NerfNetwork::density_backward input must be in column major format.");
		check(ngp_density_backward(m_, stream, ctx.get(), dL_doutput.data, dL_doutput.stride, dL_dinput ? dL_dinput->data : nullptr,
		                           dL_dinput ? dL_dinput->stride : 0, (int)mode),
		      "density_backward");
	}
};

// tcnn::NetworkWithInputEncoding (image / SDF primitives, src/testbed.cu:4101-4110)
class NetworkWithInputEncoding : public Network {
public:
	NetworkWithInputEncoding(uint32_t n_input_dims, uint32_t n_output_dims, const std::string& encoding, const std::string& network) {
		check(ngp_network_with_input_encoding_create(n_input_dims, n_output_dims, encoding.c_str(), network.c_str(), &m_),
		      "NetworkWithInputEncoding");
	}
};

// tcnn::Trainer<float, __half, __half> (src/testbed.cu:4129): owns params, gradients, optimizer state
class Trainer {
public:
	Trainer(Network& net, const std::string& optimizer, uint64_t seed = 1337) {
		check(ngp_trainer_create(net.handle(), optimizer.c_str(), seed, &t_), "Trainer");
	}
	~Trainer() { if (t_) ngp_trainer_destroy(t_); }
	Trainer(const Trainer&) = delete;
	Trainer& operator=(const Trainer&) = delete;

	void optimizer_step(void* stream, float loss_scale) {  // testbed_nerf.cu:3678
		check(ngp_trainer_optimizer_step(t_, stream, loss_scale), "optimizer_step");
	}
	uint16_t* params() const { return (uint16_t*)ngp_trainer_params(t_); }
	uint16_t* params_inference() const { return (uint16_t*)ngp_trainer_inference_params(t_); }
	uint16_t* gradients() const { return (uint16_t*)ngp_trainer_gradients(t_); }
	float* params_full_precision() const { return ngp_trainer_params_full_precision(t_); }
	uint32_t step() const { return ngp_trainer_step(t_); }
	float learning_rate() const { return ngp_trainer_learning_rate(t_); }
	void set_learning_rate(float lr) { check(ngp_trainer_set_learning_rate(t_, lr), "set_learning_rate"); }
	void set_params_full_precision(const float* host, uint64_t n) {  // src/testbed.cu:4146
		check(ngp_trainer_set_params_full_precision(t_, host, n), "set_params_full_precision");
	}
	std::vector<uint8_t> serialize() {  // src/testbed.cu:4874
		uint64_t size = 0;
		check(ngp_trainer_serialize(t_, nullptr, &size), "serialize");
		std::vector<uint8_t> b(size);
		check(ngp_trainer_serialize(t_, b.data(), &size), "serialize");
		return b;
	}
	void deserialize(const std::vector<uint8_t>& b) {  // src/testbed.cu:5040
		check(ngp_trainer_deserialize(t_, b.data(), b.size()), "deserialize");
	}
	ngp_trainer* handle() const { return t_; }

private:
	ngp_trainer* t_ = nullptr;
};

}  // namespace ngp_mi355x
