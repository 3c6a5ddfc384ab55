// testbed_host.hpp — the Testbed host (include/neural-graphics-primitives/testbed.h, src/testbed.cu) in plain
// C++17 over the engine's C-ABI (include/ngp_engine.h): mode dispatch, network (re)construction from the
// JSON config, Testbed::train / frame (headless), snapshots and the NeRF render of a camera. It holds no HIP
// code and no HIP headers: device buffers come from ngp_malloc, every kernel runs behind the C-ABI.
//
// Reference surface mirrored (names and argument meaning):
//   Testbed(mode) / load_training_data(path) / clear_training_data      testbed.cu:139-176
//   reload_network_from_file / reload_network_from_json                 testbed.cu:228-314 (parent merge)
//   reset_network(clear_density_grid)                                    testbed.cu:3903-4151
//   train(batch_size)                                                    testbed.cu:4285-4370
//   frame() (headless: train when shall_train)                           testbed.cu:3595-3761
//   n_params / n_encoding_params                                         testbed.cu:4843-4856
//   save_snapshot / load_snapshot                                        testbed.cu:4873-5057
//   set_camera_to_training_view / render_to_cpu                          testbed.cu:848-856, python_api.cu:418-427
// What lives elsewhere: decoding image files (JPEG/PNG/EXR) is the binding's job (python_api.cpp hands the
// decoded pixels to load_nerf / load_image), as the reference delegates it to stb_image / tinyexr.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ngp_engine.h"
#include "json.h"

namespace ngp_host {

using ngp::Json;

enum class ETestbedMode : int { Nerf, Sdf, Image, Volume, None };  // common.h:186-192
enum class ERenderMode : int { AO, Shade, Normals, Positions, Depth, Distortion, Cost, Slice };  // common.h:110-119

inline void check(int rc, const char* what) {
	if (rc != NGP_OK) throw std::runtime_error(std::string(what) + ": " + ngp_last_error());
}

inline bool iends_with(const std::string& s, const std::string& suffix) {
	if (s.size() < suffix.size()) return false;
	return ngp::iequals(s.substr(s.size() - suffix.size()), suffix);
}

inline bool is_directory(const std::string& p) {
	std::ifstream f(p + "/.");
	return f.good();
}

// mode_from_scene (common.cu:144-159): directories and .json are NeRF, .obj/.stl SDF, .nvdb volume, else an image
inline ETestbedMode mode_from_scene(const std::string& scene) {
	std::ifstream probe(scene);
	if (!probe.good() && !is_directory(scene)) return ETestbedMode::None;
	if (is_directory(scene) || iends_with(scene, ".json")) return ETestbedMode::Nerf;
	if (iends_with(scene, ".obj") || iends_with(scene, ".stl")) return ETestbedMode::Sdf;
	if (iends_with(scene, ".nvdb")) return ETestbedMode::Volume;
	return ETestbedMode::Image;
}

// to_string(ETestbedMode) (common.cu:175-184)
inline const char* mode_name(ETestbedMode m) {
	switch (m) {
	case ETestbedMode::Nerf: return "nerf";
	case ETestbedMode::Sdf: return "sdf";
	case ETestbedMode::Image: return "image";
	case ETestbedMode::Volume: return "volume";
	default: return "none";
	}
}

// mode_from_string (common.cu:161-173)
inline ETestbedMode mode_from_string(const std::string& s) {
	if (ngp::iequals(s, "nerf")) return ETestbedMode::Nerf;
	if (ngp::iequals(s, "sdf")) return ETestbedMode::Sdf;
	if (ngp::iequals(s, "image")) return ETestbedMode::Image;
	if (ngp::iequals(s, "volume")) return ETestbedMode::Volume;
	return ETestbedMode::None;
}

// RFC 7386 merge patch (nlohmann::json::merge_patch, the config `parent` merge of testbed.cu:95-106)
inline Json merge_patch(const Json& base, const Json& patch) {
	if (patch.type != Json::Object) return patch;
	Json out = base.type == Json::Object ? base : Json{};
	out.type = Json::Object;
	for (const auto& kv : patch.obj) {
		if (kv.second.type == Json::Null) out.obj.erase(kv.first);
		else out.obj[kv.first] = merge_patch(out.contains(kv.first) ? out.obj[kv.first] : Json{}, kv.second);
	}
	return out;
}

inline std::string read_text(const std::string& path) {
	std::ifstream f(path, std::ios::binary);
	if (!f) throw std::runtime_error("cannot open " + path);
	std::stringstream ss;
	ss << f.rdbuf();
	return ss.str();
}

// Testbed::load_network_config (testbed.cu:228-314): a config file, its "parent" merged underneath
inline Json load_network_config(const std::string& path) {
	Json cfg = Json::parse(read_text(path));
	if (cfg.contains("parent")) {
		const std::string dir = path.find('/') == std::string::npos ? "." : path.substr(0, path.rfind('/'));
		Json parent = load_network_config(dir + "/" + cfg["parent"].str);
		cfg.obj.erase("parent");
		cfg = merge_patch(parent, cfg);
	}
	return cfg;
}

// configs/<mode>/base.json of the reference fork, restated as data (nothing under the reference tree is read
// at run time); instant-ngp_amd/config.py holds the same dicts (tests/test_pyngp.py checks they agree)
inline std::string default_network_config(ETestbedMode mode) {
	switch (mode) {
	case ETestbedMode::Nerf:  // configs/nerf/base.json (fork: L=4, F=4, T=2^19)
		return R"({"loss": {"otype": "Huber"},
 "optimizer": {"otype": "Ema", "decay": 0.95, "nested": {"otype": "ExponentialDecay", "decay_start": 20000,
   "decay_interval": 10000, "decay_base": 0.33, "nested": {"otype": "Adam", "learning_rate": 1e-2, "beta1": 0.9,
   "beta2": 0.99, "epsilon": 1e-15, "l2_reg": 1e-6}}},
 "encoding": {"otype": "HashGrid", "n_levels": 4, "n_features_per_level": 4, "log2_hashmap_size": 19, "base_resolution": 16},
 "network": {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": 64, "n_hidden_layers": 1},
 "dir_encoding": {"otype": "Composite", "nested": [{"n_dims_to_encode": 3, "otype": "SphericalHarmonics", "degree": 4},
   {"otype": "Identity"}]},
 "rgb_network": {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": 64, "n_hidden_layers": 2}})";
	case ETestbedMode::Sdf:  // configs/sdf/base.json
		return R"({"loss": {"otype": "MAPE"},
 "optimizer": {"otype": "Ema", "decay": 0.95, "nested": {"otype": "ExponentialDecay", "decay_start": 10000,
   "decay_interval": 5000, "decay_base": 0.33, "nested": {"otype": "Adam", "learning_rate": 1e-4, "beta1": 0.9,
   "beta2": 0.99, "epsilon": 1e-15, "l2_reg": 1e-6}}},
 "encoding": {"otype": "HashGrid", "n_levels": 16, "n_features_per_level": 2, "log2_hashmap_size": 19, "base_resolution": 16},
 "network": {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": 64, "n_hidden_layers": 2}})";
	case ETestbedMode::Image:  // configs/image/base.json
		return R"({"loss": {"otype": "L2"},
 "optimizer": {"otype": "ExponentialDecay", "decay_start": 20000, "decay_interval": 10000, "decay_base": 0.33,
   "nested": {"otype": "Adam", "learning_rate": 1e-2, "beta1": 0.9, "beta2": 0.99, "epsilon": 1e-15, "l2_reg": 1e-6}},
 "encoding": {"otype": "HashGrid", "n_levels": 16, "n_features_per_level": 2, "log2_hashmap_size": 24, "base_resolution": 16},
 "network": {"otype": "FullyFusedMLP", "activation": "ReLU", "output_activation": "None", "n_neurons": 64, "n_hidden_layers": 2}})";
	default:
		throw std::runtime_error("no network config for this mode (volume rendering is out of scope, SURVEY §2)");
	}
}

// OBJ triangle soup (tinyobjloader's role in Testbed::load_mesh, testbed_sdf.cu:1120): vertices of every
// face, fans triangulated; returns [3T x 3] floats
inline std::vector<float> read_obj_triangles(const std::string& path) {
	std::ifstream f(path);
	if (!f) throw std::runtime_error("cannot open " + path);
	std::vector<float> v, out;
	std::string line;
	while (std::getline(f, line)) {
		std::istringstream ls(line);
		std::string tag;
		ls >> tag;
		if (tag == "v") {
			float x, y, z;
			ls >> x >> y >> z;
			v.insert(v.end(), {x, y, z});
		} else if (tag == "f") {
			std::vector<long> idx;
			std::string tok;
			while (ls >> tok) {
				long i = std::stol(tok.substr(0, tok.find('/')));
				idx.push_back(i < 0 ? (long)(v.size() / 3) + i : i - 1);
			}
			for (size_t k = 2; k < idx.size(); ++k)
				for (long i : {idx[0], idx[k - 1], idx[k]}) {
					if (i < 0 || (size_t)i * 3 + 2 >= v.size()) throw std::runtime_error("obj: face index out of range");
					out.insert(out.end(), {v[i * 3], v[i * 3 + 1], v[i * 3 + 2]});
				}
		}
	}
	if (out.empty()) throw std::runtime_error("obj: no triangles in " + path);
	return out;
}

inline float half_to_float(uint16_t h) {
	const uint32_t s = (h >> 15) & 1, e = (h >> 10) & 31, m = h & 1023;
	float v;
	if (e == 0) v = std::ldexp((float)m, -24);
	else if (e == 31) v = m ? NAN : INFINITY;
	else v = std::ldexp((float)(m | 1024), (int)e - 25);
	return s ? -v : v;
}
inline float linear_to_srgb(float x) { return x < 0.0031308f ? 12.92f * x : 1.055f * std::pow(std::max(x, 0.f), 0.41666f) - 0.055f; }
inline float srgb_to_linear(float x) { return x <= 0.04045f ? x / 12.92f : std::pow((x + 0.055f) / 1.055f, 2.4f); }

struct DeviceBuffer {
	void* p = nullptr;
	size_t bytes = 0;
	DeviceBuffer() = default;
	DeviceBuffer(const DeviceBuffer&) = delete;
	DeviceBuffer& operator=(const DeviceBuffer&) = delete;
	~DeviceBuffer() { if (p) ngp_free(p); }
	template <typename T> T* get(size_t n) {
		const size_t b = n * sizeof(T);
		if (b > bytes) {
			if (p) ngp_free(p);
			p = nullptr;
			check(ngp_malloc(&p, b), "ngp_malloc");
			bytes = b;
		}
		return (T*)p;
	}
};

class Testbed {
public:
	explicit Testbed(ETestbedMode mode = ETestbedMode::None) { set_mode(mode); }
	~Testbed() { free_network(); free_data(); }
	Testbed(const Testbed&) = delete;
	Testbed& operator=(const Testbed&) = delete;

	// ---- mode and configuration -------------------------------------------------------------------
	ETestbedMode mode() const { return m_testbed_mode; }
	// Testbed::set_mode (testbed.cu:178-226): a new mode drops the network, the data and the config
	void set_mode(ETestbedMode mode) {
		if (mode == m_testbed_mode && m_mode_set) return;
		free_network();
		free_data();
		m_testbed_mode = mode;
		m_mode_set = true;
		m_training_step = 0;
		m_network_config = mode == ETestbedMode::None || mode == ETestbedMode::Volume ? Json{}
		                                                                                 : Json::parse(default_network_config(mode));
	}
	void reload_network_from_json(const std::string& json_text) {
		m_network_config = Json::parse(json_text);
		reset_network();
	}
	void reload_network_from_file(const std::string& path) {
		if (!path.empty()) m_network_config = load_network_config(path);
		else if (m_network_config.type != Json::Object) m_network_config = Json::parse(default_network_config(m_testbed_mode));
		reset_network();
	}
	std::string network_config() const { return m_network_config.dump(); }

	// ---- training data ------------------------------------------------------------------------------
	// Testbed::load_nerf + load_nerf_post (testbed_nerf.cu:3093-3109): decoded images (RGBA8 sRGB) with their
	// metadata after nerf_matrix_to_ngp, and the dataset's aabb_scale
	void load_nerf(const std::vector<ngp_nerf_image>& images, const std::vector<const void*>& rgba8, float aabb_scale,
	               float dataset_scale = 1.0f) {
		set_mode(ETestbedMode::Nerf);
		if (images.empty() || images.size() != rgba8.size()) throw std::runtime_error("load_nerf: one RGBA8 buffer per image");
		free_network();
		free_data();
		check(ngp_nerf_dataset_create((uint32_t)images.size(), images.data(), rgba8.data(), &m_nerf_dataset), "ngp_nerf_dataset_create");
		m_nerf_images = images;
		m_aabb_scale = aabb_scale;
		m_dataset_scale = dataset_scale;  // NerfDataset::scale (nerf_loader.cu:388): Depth renders in its units
		check(ngp_nerf_default_config(aabb_scale, &m_nerf_cfg), "ngp_nerf_default_config");
		m_training_data_available = true;
		set_camera_to_training_view(0);
	}
	// Testbed::load_image (testbed_image.cu:372-402): RGBA float [h x w x 4], linear colours
	void load_image(uint32_t width, uint32_t height, const float* rgba) {
		set_mode(ETestbedMode::Image);
		free_network();
		free_data();
		check(ngp_image_create(width, height, rgba, &m_image), "ngp_image_create");
		check(ngp_image_default_config(&m_image_cfg), "ngp_image_default_config");
		m_image_res[0] = width;
		m_image_res[1] = height;
		m_training_data_available = true;
	}
	// Testbed::load_mesh (testbed_sdf.cu:1120-1165): triangle soup [3T x 3] normalised into the unit cube
	void load_mesh(const std::vector<float>& vertices) {
		set_mode(ETestbedMode::Sdf);
		free_network();
		free_data();
		const size_t nv = vertices.size() / 3;
		if (nv == 0 || nv % 3 != 0) throw std::runtime_error("load_mesh: vertices must hold whole triangles");
		float lo[3], hi[3];
		for (int d = 0; d < 3; ++d) { lo[d] = INFINITY; hi[d] = -INFINITY; }
		for (size_t i = 0; i < nv; ++i)
			for (int d = 0; d < 3; ++d) { lo[d] = std::min(lo[d], vertices[i * 3 + d]); hi[d] = std::max(hi[d], vertices[i * 3 + d]); }
		const float inflation = 0.005f;
		auto norm = [](const float* a, const float* b) {
			float s = 0.f;
			for (int d = 0; d < 3; ++d) s += (b[d] - a[d]) * (b[d] - a[d]);
			return std::sqrt(s);
		};
		float amount = norm(lo, hi) * inflation;
		for (int d = 0; d < 3; ++d) { lo[d] -= amount; hi[d] += amount; }
		float diag[3], scale = 0.f;
		for (int d = 0; d < 3; ++d) { diag[d] = hi[d] - lo[d]; scale = std::max(scale, diag[d]); }
		std::vector<float> tris(vertices.size());
		float alo[3], ahi[3];
		for (int d = 0; d < 3; ++d) { alo[d] = INFINITY; ahi[d] = -INFINITY; }
		for (size_t i = 0; i < nv; ++i)
			for (int d = 0; d < 3; ++d) {
				const float v = (vertices[i * 3 + d] - lo[d] - 0.5f * diag[d]) / scale + 0.5f;
				tris[i * 3 + d] = v;
				alo[d] = std::min(alo[d], v);
				ahi[d] = std::max(ahi[d], v);
			}
		amount = norm(alo, ahi) * inflation;
		for (int d = 0; d < 3; ++d) {
			m_sdf_aabb_min[d] = std::max(alo[d] - amount, 0.f);
			m_sdf_aabb_max[d] = std::min(ahi[d] + amount, 1.f);
		}
		m_bounding_radius = std::sqrt(0.75f);
		check(ngp_sdf_mesh_create((uint32_t)(nv / 3), tris.data(), &m_sdf_mesh), "ngp_sdf_mesh_create");
		m_training_data_available = true;
	}
	void load_mesh_file(const std::string& path) { load_mesh(read_obj_triangles(path)); }
	void clear_training_data() {
		free_network();
		free_data();
	}
	bool training_data_available() const { return m_training_data_available; }

	// ---- network ------------------------------------------------------------------------------------
	// Testbed::reset_network (testbed.cu:3903-4151): the model from the config sections, a trainer seeded
	// from m_seed, and for NeRF the training state (density grid, counters, rng). reset_density_grid = false
	// keeps the occupancy grid of the previous network.
	void reset_network(bool reset_density_grid = true) {
		if (m_testbed_mode == ETestbedMode::None) throw std::runtime_error("reset_network: no mode");
		if (m_testbed_mode == ETestbedMode::Volume) throw std::runtime_error("the volume primitive is out of scope (SURVEY §2)");
		std::vector<float> kept_grid;
		if (!reset_density_grid && m_nerf_trainer) {
			const float* g = nullptr;
			const uint8_t* b = nullptr;
			const float* m = nullptr;
			check(ngp_nerf_trainer_buffers_read(m_nerf_trainer, &g, &b, &m), "ngp_nerf_trainer_buffers_read");
			kept_grid.resize((size_t)128 * 128 * 128 * (m_nerf_cfg.max_cascade + 1));
			check(ngp_memcpy(kept_grid.data(), g, kept_grid.size() * 4, 2 /* device to host */), "ngp_memcpy");
		}
		free_network();
		m_training_step = 0;
		m_loss_scalar = 0.f;
		// testbed.cu:3975-3997: a missing base_resolution becomes 2^(log2_hashmap_size / n_pos) and is written
		// into the config. per_level_scale: the fork sets only its log member to 2.0 (:3991), so the auto-scale
		// branch never runs and the encoding config reaches the network unchanged (:4037): a config's own value
		// stays (configs/nerf/densegrid.json 1.405), an absent key is tcnn's default 2.0 (parse_grid)
		Json enc = m_network_config["encoding"];
		const uint32_t n_pos = m_testbed_mode == ETestbedMode::Image ? 2u : 3u;
		if (enc.number_or("base_resolution", 0.0) == 0.0) {
			enc.obj["base_resolution"].type = Json::Number;
			enc.obj["base_resolution"].num = (double)(1u << ((uint32_t)enc.number_or("log2_hashmap_size", 15.0) / n_pos));
		}
		const std::string opt = m_network_config["optimizer"].dump();
		switch (m_testbed_mode) {
		case ETestbedMode::Nerf: {
			const Json& c = m_network_config;
			check(ngp_nerf_network_create(3, 3, 0, 4, enc.dump().c_str(), c.contains("dir_encoding") ? c["dir_encoding"].dump().c_str() : nullptr,
			                              c["network"].dump().c_str(), c["rgb_network"].dump().c_str(), &m_model),
			      "ngp_nerf_network_create");
			break;
		}
		case ETestbedMode::Image:
			check(ngp_network_with_input_encoding_create(2, 3, enc.dump().c_str(), m_network_config["network"].dump().c_str(), &m_model),
			      "ngp_network_with_input_encoding_create");
			break;
		case ETestbedMode::Sdf:
			check(ngp_network_with_input_encoding_create(3, 1, enc.dump().c_str(), m_network_config["network"].dump().c_str(), &m_model),
			      "ngp_network_with_input_encoding_create");
			break;
		default: break;
		}
		check(ngp_trainer_create(m_model, opt.c_str(), m_seed, &m_trainer), "ngp_trainer_create");
		m_rng = host_pcg32(m_seed);
		if (m_testbed_mode == ETestbedMode::Nerf && m_nerf_dataset) {
			check(ngp_nerf_trainer_create(m_model, m_trainer, m_nerf_dataset, &m_nerf_cfg, m_seed, &m_nerf_trainer),
			      "ngp_nerf_trainer_create");
			if (!kept_grid.empty()) {
				float* g = nullptr;
				uint8_t* b = nullptr;
				float* m = nullptr;
				check(ngp_nerf_trainer_buffers(m_nerf_trainer, &g, &b, &m), "ngp_nerf_trainer_buffers");
				check(ngp_memcpy(g, kept_grid.data(), kept_grid.size() * 4, 1 /* host to device */), "ngp_memcpy");
			}
		}
	}
	uint64_t n_params() const { return m_model ? ngp_model_n_params(m_model) : 0; }
	uint64_t n_encoding_params() const {
		if (!m_model) return 0;
		ngp_param_layout lo;
		check(ngp_model_param_layout(m_model, &lo), "ngp_model_param_layout");
		return lo.grid_params;
	}

	// ---- training -----------------------------------------------------------------------------------
	// Testbed::train (testbed.cu:4285-4370); the loss is read back every 16 steps, as the reference does
	void train(uint32_t batch_size) {
		if (!m_training_data_available) {
			m_train = false;
			return;
		}
		if (m_testbed_mode == ETestbedMode::None) throw std::runtime_error("Cannot train without a mode.");
		if (!m_trainer) reset_network();
		const bool get_loss = m_training_step % 16 == 0;
		switch (m_testbed_mode) {
		case ETestbedMode::Nerf: {
			if (batch_size != m_nerf_cfg.target_batch_size) {
				m_nerf_cfg.target_batch_size = batch_size;
				push_nerf_config();
			}
			ngp_nerf_stats st;
			check(ngp_nerf_train_step(m_nerf_trainer, nullptr, get_loss ? 1 : 0, &st), "ngp_nerf_train_step");
			if (get_loss) m_loss_scalar = st.loss;
			m_training_step = st.step;
			return;
		}
		case ETestbedMode::Image: {
			float* loss = m_loss_dev.get<float>(1);
			if (get_loss) check(ngp_memcpy(loss, &ZERO, 4, 1), "ngp_memcpy");
			check(ngp_image_train_step(m_image, m_trainer, nullptr, batch_size, &m_rng, &m_image_cfg, get_loss ? loss : nullptr),
			      "ngp_image_train_step");
			break;
		}
		case ETestbedMode::Sdf: {
			const uint32_t n = batch_size / 8 * 8;
			float* pos = m_sdf_pos.get<float>((size_t)n * 3);
			float* dist = m_sdf_dist.get<float>(n);
			float* pos_s = m_sdf_pos_s.get<float>((size_t)n * 3);
			float* dist_s = m_sdf_dist_s.get<float>(n);
			float* loss = m_loss_dev.get<float>(1);
			if (get_loss) check(ngp_memcpy(loss, &ZERO, 4, 1), "ngp_memcpy");
			// generate_sdf_data_online (testbed.h:842): the batch is regenerated every step
			if (m_sdf_generate_online || m_training_step == 0) {
				const float stddev = m_bounding_radius / 1024.0f * m_sdf_surface_offset_scale;
				check(ngp_sdf_generate_training_samples(m_sdf_mesh, nullptr, n, &m_rng, m_sdf_aabb_min, m_sdf_aabb_max, stddev, pos, dist),
				      "ngp_sdf_generate_training_samples");
			}
			check(ngp_sdf_train_step(m_trainer, nullptr, n, pos, dist, m_training_step, pos_s, dist_s, get_loss ? loss : nullptr),
			      "ngp_sdf_train_step");
			break;
		}
		default: throw std::runtime_error("Invalid training mode.");
		}
		check(ngp_stream_synchronize(nullptr), "ngp_stream_synchronize");
		if (get_loss) {
			float l = 0.f;
			check(ngp_memcpy(&l, m_loss_dev.p, 4, 2), "ngp_memcpy");
			m_loss_scalar = l;
		}
		++m_training_step;
	}
	// Testbed::frame (testbed.cu:3595-3761) without a window: train_and_render trains when shall_train
	bool frame() {
		if (m_train) train(m_training_batch_size);
		return true;
	}
	float loss() const { return m_loss_scalar; }
	uint32_t training_step() const { return m_training_step; }

	// ---- snapshots (the .ingp / msgpack format of testbed.cu:4873-5057, every mode) -----------------------
	void save_snapshot(const std::string& path, bool include_optimizer_state, bool compress) {
		if (m_testbed_mode == ETestbedMode::Nerf) {
			require_nerf_trainer("save_snapshot");
			check(ngp_nerf_save_snapshot(m_nerf_trainer, nullptr, path.c_str(), m_network_config.dump().c_str(),
			                             include_optimizer_state ? 1 : 0, compress ? 1 : 0),
			      "ngp_nerf_save_snapshot");
			return;
		}
		if (!m_trainer) throw std::runtime_error("save_snapshot: no network (train first)");
		const float img_min[3] = {0.f, 0.f, 0.f}, img_max[3] = {1.f, 1.f, 1.f};
		const bool sdf = m_testbed_mode == ETestbedMode::Sdf;
		check(ngp_save_snapshot(m_trainer, nullptr, path.c_str(), m_network_config.dump().c_str(), mode_name(m_testbed_mode),
		                        sdf ? m_sdf_aabb_min : img_min, sdf ? m_sdf_aabb_max : img_max, m_bounding_radius, m_training_step,
		                        m_loss_scalar, include_optimizer_state ? 1 : 0, compress ? 1 : 0),
		      "ngp_save_snapshot");
	}
	// Testbed::load_snapshot (testbed.cu:4939-5057): the snapshot's mode (a different one drops the loaded data, as
	// set_mode does), its network config, then the trainer state and the mode's members
	void load_snapshot(const std::string& path) {
		char mode[32];
		check(ngp_snapshot_mode(path.c_str(), mode, sizeof mode), "ngp_snapshot_mode");
		const ETestbedMode m = mode_from_string(mode);
		if (m == ETestbedMode::None || m == ETestbedMode::Volume)
			throw std::runtime_error(std::string("load_snapshot: unsupported snapshot mode '") + mode + "'");
		set_mode(m);
		if (m == ETestbedMode::Nerf && !m_nerf_dataset)
			throw std::runtime_error("load_snapshot: load the NeRF training data first (the snapshot's dataset member is not read)");
		uint64_t size = 0;
		check(ngp_snapshot_network_config(path.c_str(), nullptr, &size), "ngp_snapshot_network_config");
		std::string cfg(size, '\0');
		check(ngp_snapshot_network_config(path.c_str(), &cfg[0], &size), "ngp_snapshot_network_config");
		cfg.resize(strlen(cfg.c_str()));
		m_network_config = Json::parse(cfg);
		reset_network();
		if (m == ETestbedMode::Nerf) {
			check(ngp_nerf_load_snapshot(m_nerf_trainer, nullptr, path.c_str()), "ngp_nerf_load_snapshot");
			m_training_step = ngp_trainer_step(m_trainer);  // one optimizer step per training step
			return;
		}
		float amin[3], amax[3];
		check(ngp_load_snapshot(m_trainer, nullptr, path.c_str(), &m_training_step, &m_loss_scalar, amin, amax, &m_bounding_radius),
		      "ngp_load_snapshot");
		if (m == ETestbedMode::Sdf) {
			std::memcpy(m_sdf_aabb_min, amin, sizeof amin);
			std::memcpy(m_sdf_aabb_max, amax, sizeof amax);
		}
	}

	// ---- camera and rendering -----------------------------------------------------------------------
	// set_camera_to_training_view (testbed.cu:848-856): the view's camera, relative focal length and screen centre
	void set_camera_to_training_view(uint32_t i) {
		if (i >= m_nerf_images.size()) throw std::runtime_error("set_camera_to_training_view: no such training view");
		const ngp_nerf_image& im = m_nerf_images[i];
		std::memcpy(m_camera, im.xform, sizeof(m_camera));
		const float res_axis = (float)(m_fov_axis == 0 ? im.width : im.height);
		m_relative_focal_length[0] = im.focal_length[0] / res_axis;
		m_relative_focal_length[1] = im.focal_length[1] / res_axis;
		m_screen_center[0] = 1.0f - im.principal_point[0];
		m_screen_center[1] = 1.0f - im.principal_point[1];
		m_lens_mode = im.lens_mode;
		std::memcpy(m_lens_params, im.lens_params, sizeof(m_lens_params));
		m_training_view = i;
	}
	uint32_t n_training_views() const { return (uint32_t)m_nerf_images.size(); }
	// render_to_cpu (python_api.cu:418-427): an RGBA float image [height x width x 4], linear colours or sRGB.
	// NeRF: the NerfTracer over the occupancy bitfield with the inference (EMA) parameters, spp samples
	// averaged; Image: the network evaluated at the pixel centres.
	std::vector<float> render(uint32_t width, uint32_t height, uint32_t spp, bool linear) {
		if (width == 0 || height == 0 || spp == 0) throw std::runtime_error("render: empty image");
		if (!m_model) throw std::runtime_error("render: no network (train or load a snapshot first)");
		std::vector<float> out((size_t)width * height * 4);
		if (m_testbed_mode == ETestbedMode::Nerf) {
			if ((int)m_render_mode > (int)ERenderMode::Depth)
				throw std::runtime_error("render: ERenderMode AO, Shade, Normals, Positions and Depth are implemented");
			require_nerf_trainer("render");
			if (!m_renderer) check(ngp_nerf_renderer_create(&m_renderer), "ngp_nerf_renderer_create");
			check(ngp_nerf_renderer_set_mode(m_renderer, (int)m_render_mode), "ngp_nerf_renderer_set_mode");
			// depth_scale = 1 / m_nerf.training.dataset.scale (render_nerf, testbed_nerf.cu:2822)
			check(ngp_nerf_renderer_set_depth_scale(m_renderer, 1.0f / m_dataset_scale), "ngp_nerf_renderer_set_depth_scale");
			ngp_nerf_image cam{};
			cam.width = width;
			cam.height = height;
			const float res_axis = (float)(m_fov_axis == 0 ? width : height);
			cam.focal_length[0] = m_relative_focal_length[0] * res_axis * m_zoom;
			cam.focal_length[1] = m_relative_focal_length[1] * res_axis * m_zoom;
			cam.principal_point[0] = 1.0f - m_screen_center[0];
			cam.principal_point[1] = 1.0f - m_screen_center[1];
			std::memcpy(cam.xform, m_camera, sizeof(m_camera));
			cam.lens_mode = m_render_with_lens_distortion ? m_lens_mode : 0;
			std::memcpy(cam.lens_params, m_lens_params, sizeof(m_lens_params));
			const float* g = nullptr;
			const uint8_t* bf = nullptr;
			const float* mean = nullptr;
			check(ngp_nerf_trainer_buffers_read(m_nerf_trainer, &g, &bf, &mean), "ngp_nerf_trainer_buffers_read");
			float* dev = m_render_buf.get<float>(out.size());
			ngp_nerf_config cfg = m_nerf_cfg;
			check(ngp_nerf_render(m_renderer, m_model, &cfg, nullptr, &cam, bf, spp, m_render_sample_index, m_render_min_transmittance,
			                      m_background_color, 1, dev),
			      "ngp_nerf_render");
			check(ngp_memcpy(out.data(), dev, out.size() * 4, 2), "ngp_memcpy");
		} else if (m_testbed_mode == ETestbedMode::Image) {
			const size_t n = (size_t)width * height;
			std::vector<float> pos(n * 2);
			for (uint32_t y = 0; y < height; ++y)
				for (uint32_t x = 0; x < width; ++x) {
					pos[((size_t)y * width + x) * 2] = (x + 0.5f) / width;
					pos[((size_t)y * width + x) * 2 + 1] = (y + 0.5f) / height;
				}
			float* dpos = m_render_buf.get<float>(n * 2);
			check(ngp_memcpy(dpos, pos.data(), n * 8, 1), "ngp_memcpy");
			uint16_t* dout = m_render_out.get<uint16_t>(n * 16);
			check(ngp_inference(m_model, nullptr, (uint32_t)n, dpos, 2, dout, 16, NGP_LAYOUT_AOS, 1), "ngp_inference");
			std::vector<uint16_t> h(n * 16);
			check(ngp_memcpy(h.data(), dout, n * 32, 2), "ngp_memcpy");
			for (size_t i = 0; i < n; ++i) {
				for (int c = 0; c < 3; ++c) {
					float v = half_to_float(h[i * 16 + c]);
					// the network regresses sRGB targets unless linear_colors (testbed_image.cu:167-212)
					out[i * 4 + c] = m_image_cfg.linear_colors ? v : srgb_to_linear(v);
				}
				out[i * 4 + 3] = 1.0f;
			}
		} else {
			throw std::runtime_error("render: SDF sphere tracing and volume rendering are out of scope (SURVEY §2)");
		}
		if (!linear)
			for (size_t i = 0; i < out.size(); i += 4)
				for (int c = 0; c < 3; ++c) out[i + c] = linear_to_srgb(out[i + c]);
		return out;
	}

	// NeRF training knobs (Testbed::Nerf::Training, testbed.h:716-785) reach a live trainer here
	ngp_nerf_config& nerf_config() { return m_nerf_cfg; }
	void push_nerf_config() {
		if (m_nerf_trainer) check(ngp_nerf_trainer_set_config(m_nerf_trainer, &m_nerf_cfg), "ngp_nerf_trainer_set_config");
	}
	ngp_image_config& image_config() { return m_image_cfg; }
	const std::vector<ngp_nerf_image>& nerf_images() const { return m_nerf_images; }
	float aabb_scale() const { return m_aabb_scale; }
	ngp_trainer* trainer() const { return m_trainer; }
	ngp_model* model() const { return m_model; }

	// public members with the reference's names (testbed.h)
	bool m_train = false;
	uint32_t m_training_batch_size = 1u << 18;
	uint32_t m_seed = 1337;
	float m_background_color[4] = {0.f, 0.f, 0.f, 1.f};
	ERenderMode m_render_mode = ERenderMode::Shade;
	float m_camera[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0.5f, 0.5f, -1.5f};  // mat4x3, column-major
	float m_relative_focal_length[2] = {1.0f, 1.0f};
	float m_screen_center[2] = {0.5f, 0.5f};
	uint32_t m_fov_axis = 1;
	float m_zoom = 1.0f;
	uint32_t m_render_sample_index = 0;
	float m_render_min_transmittance = 0.01f;   // Nerf::render_min_transmittance (testbed.h)
	bool m_render_with_lens_distortion = false;  // Nerf::render_with_lens_distortion
	bool m_sdf_generate_online = true;           // Sdf::Training::generate_sdf_data_online (testbed.h:842)
	float m_sdf_surface_offset_scale = 1.0f;     // Sdf::Training::surface_offset_scale
	float m_bounding_radius = 1.0f;
	uint32_t m_training_view = 0;

private:
	static constexpr float ZERO = 0.f;
	static ngp_rng host_pcg32(uint64_t seed) {  // tcnn::pcg32(initstate, initseq = 1)
		const uint64_t mult = 0x5851F42D4C957F2DULL;
		ngp_rng r;
		r.inc = (1ull << 1) | 1u;
		r.state = 0;
		r.state = r.state * mult + r.inc;
		r.state += seed;
		r.state = r.state * mult + r.inc;
		return r;
	}
	void require_nerf_trainer(const char* what) {
		if (m_testbed_mode != ETestbedMode::Nerf) throw std::runtime_error(std::string(what) + ": not a NeRF testbed");
		if (!m_nerf_trainer) {
			if (!m_nerf_dataset) throw std::runtime_error(std::string(what) + ": no NeRF training data loaded");
			reset_network();
		}
	}
	void free_network() {
		if (m_nerf_trainer) ngp_nerf_trainer_destroy(m_nerf_trainer);
		if (m_trainer) ngp_trainer_destroy(m_trainer);
		if (m_model) ngp_model_destroy(m_model);
		m_nerf_trainer = nullptr;
		m_trainer = nullptr;
		m_model = nullptr;
	}
	void free_data() {
		if (m_renderer) ngp_nerf_renderer_destroy(m_renderer);
		if (m_nerf_dataset) ngp_nerf_dataset_destroy(m_nerf_dataset);
		if (m_image) ngp_image_destroy(m_image);
		if (m_sdf_mesh) ngp_sdf_mesh_destroy(m_sdf_mesh);
		m_renderer = nullptr;
		m_nerf_dataset = nullptr;
		m_image = nullptr;
		m_sdf_mesh = nullptr;
		m_nerf_images.clear();
		m_training_data_available = false;
	}

	ETestbedMode m_testbed_mode = ETestbedMode::None;
	bool m_mode_set = false;
	Json m_network_config;
	bool m_training_data_available = false;
	uint32_t m_training_step = 0;
	float m_loss_scalar = 0.f;
	ngp_rng m_rng{};
	ngp_model* m_model = nullptr;
	ngp_trainer* m_trainer = nullptr;
	// NeRF
	ngp_nerf_dataset* m_nerf_dataset = nullptr;
	ngp_nerf_trainer* m_nerf_trainer = nullptr;
	ngp_nerf_renderer* m_renderer = nullptr;
	ngp_nerf_config m_nerf_cfg{};
	std::vector<ngp_nerf_image> m_nerf_images;
	float m_aabb_scale = 1.f;
	float m_dataset_scale = 1.f;
	uint32_t m_lens_mode = 0;
	float m_lens_params[4] = {0, 0, 0, 0};
	// image
	ngp_image* m_image = nullptr;
	ngp_image_config m_image_cfg{};
	uint32_t m_image_res[2] = {0, 0};
	// SDF
	ngp_sdf_mesh* m_sdf_mesh = nullptr;
	float m_sdf_aabb_min[3] = {0, 0, 0}, m_sdf_aabb_max[3] = {1, 1, 1};
	DeviceBuffer m_sdf_pos, m_sdf_dist, m_sdf_pos_s, m_sdf_dist_s;
	DeviceBuffer m_loss_dev, m_render_buf, m_render_out;
};

}  // namespace ngp_host
