// python_api.cpp — the `pyngp` pybind11 module (src/python_api.cpp of the reference, :258-698): the Testbed
// host of testbed_host.hpp with the reference's Python names and argument meaning, over the engine's C-ABI.
// Built by g++ against libngp_engine.so (no HIP headers); scripts use it as the reference's do
// (`import pyngp as ngp`, scripts/run.py:25): ngp.Testbed(), load_training_data, shall_train, frame / train,
// training_step, loss, save_snapshot / load_snapshot, render.
//
// Headless: no window, GUI, DLSS or VR members (SURVEY §2 out of scope). Image files are decoded by the
// package's Python readers (nerf_data.load_nerf: PIL for JPEG/PNG; exr.read_exr), the way the reference
// hands decoding to stb_image / tinyexr; everything after decoding runs in C++ and on the GPU.
#include <pybind11/eval.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "testbed_host.hpp"

namespace py = pybind11;
using namespace ngp_host;

namespace {

enum class ELossType : int { L2, L1, Mape, Smape, Huber, LogL1, RelativeL2 };  // common.h (python_api.cu:306-315)
enum class ENerfActivation : int { None, ReLU, Logistic, Exponential };       // nerf.h (python_api.cu:323-328)
enum class ERandomMode : int { Random = 0, Stratified = 3 };                   // common.h:124-130 (engine's subset)

std::string g_module_file;

// instant-ngp_amd/ as the Python package `instant_ngp_amd` (its directory name is not an identifier); this
// module lives in instant-ngp_amd/lib/
py::object package() {
	py::object modules = py::module_::import("sys").attr("modules");
	if (modules.contains("instant_ngp_amd")) return modules["instant_ngp_amd"];
	py::dict scope;
	scope["module_file"] = g_module_file;
	py::exec(R"(
import importlib.util, os, sys
pkg_dir = os.path.dirname(os.path.dirname(os.path.abspath(module_file)))
spec = importlib.util.spec_from_file_location("instant_ngp_amd", os.path.join(pkg_dir, "__init__.py"),
                                              submodule_search_locations=[pkg_dir])
mod = importlib.util.module_from_spec(spec)
sys.modules["instant_ngp_amd"] = mod
spec.loader.exec_module(mod)
)", scope);
	return modules["instant_ngp_amd"];
}

// Testbed::load_training_data (testbed.cu:139-165): the mode follows the scene (mode_from_scene)
void load_training_data(Testbed& tb, const std::string& path) {
	const ETestbedMode mode = mode_from_scene(path);
	switch (mode) {
	case ETestbedMode::Nerf: {
		py::object d = package().attr("nerf_data").attr("load_nerf")(path);
		py::list images = d.attr("images"), pixels = d.attr("rgba8");
		py::object ctypes = py::module_::import("ctypes");
		std::vector<ngp_nerf_image> meta(py::len(images));
		std::vector<py::array_t<uint8_t, py::array::c_style | py::array::forcecast>> keep;
		std::vector<const void*> ptrs;
		for (size_t i = 0; i < meta.size(); ++i) {
			py::object im = images[i];
			if (ctypes.attr("sizeof")(im).cast<size_t>() != sizeof(ngp_nerf_image))
				throw std::runtime_error("load_training_data: NerfImage layout differs from ngp_nerf_image");
			std::memcpy(&meta[i], (const void*)ctypes.attr("addressof")(im).cast<uintptr_t>(), sizeof(ngp_nerf_image));
			keep.emplace_back(pixels[i]);
			if (keep.back().ndim() != 3 || (uint32_t)keep.back().shape(0) != meta[i].height ||
			    (uint32_t)keep.back().shape(1) != meta[i].width || keep.back().shape(2) != 4)
				throw std::runtime_error("load_training_data: image buffer shape does not match its metadata");
			ptrs.push_back(keep.back().data());
		}
		const float aabb_scale = d.attr("aabb_scale").cast<float>();
		const float scale = py::hasattr(d, "scale") ? d.attr("scale").cast<float>() : 1.0f;
		py::gil_scoped_release nogil;
		tb.load_nerf(meta, ptrs, aabb_scale, scale);
		break;
	}
	case ETestbedMode::Image: {
		py::object arr;
		if (iends_with(path, ".exr")) arr = package().attr("exr").attr("read_exr")(path);
		else if (iends_with(path, ".npy")) arr = py::module_::import("numpy").attr("load")(path);
		else throw std::runtime_error("load_training_data: images are read from .exr or .npy [H, W, 4] float files");
		py::array_t<float, py::array::c_style | py::array::forcecast> a(arr);
		if (a.ndim() != 3 || a.shape(2) != 4) throw std::runtime_error("load_training_data: expected an [H, W, 4] RGBA image");
		tb.load_image((uint32_t)a.shape(1), (uint32_t)a.shape(0), a.data());
		break;
	}
	case ETestbedMode::Sdf: {
		py::gil_scoped_release nogil;
		tb.load_mesh_file(path);
		break;
	}
	case ETestbedMode::Volume: throw std::runtime_error("the volume primitive is out of scope (SURVEY §2)");
	default: throw std::runtime_error("Unknown scene format for path '" + path + "'.");
	}
}

// Testbed::load_file (testbed.cu:316-375): snapshots, network configs, else training data
void load_file(Testbed& tb, const std::string& path) {
	if (iends_with(path, ".ingp") || iends_with(path, ".msgpack")) {
		tb.load_snapshot(path);
		return;
	}
	if (iends_with(path, ".json") && !is_directory(path)) {
		const Json j = Json::parse(read_text(path));
		if (j.contains("encoding") || j.contains("network") || j.contains("parent")) {
			tb.reload_network_from_file(path);
			return;
		}
	}
	const bool had_data = tb.training_data_available();
	load_training_data(tb, path);
	if (!had_data) tb.m_train = true;  // testbed.cu:363-371
}

// views of the Testbed's nested members (Testbed::Nerf, ::Sdf, ::Image and their ::Training)
struct NerfView { Testbed* t; };
struct NerfTrainingView { Testbed* t; };
struct NerfDatasetView { Testbed* t; };
struct SdfView { Testbed* t; };
struct SdfTrainingView { Testbed* t; };
struct ImageView { Testbed* t; };
struct ImageTrainingView { Testbed* t; };

// a Testbed::Nerf::Training knob: written into the trainer's live configuration (ngp_nerf_trainer_set_config)
template <typename V, typename T>
void nerf_knob(py::class_<V>& c, const char* name, T ngp_nerf_config::*field) {
	c.def_property(name, [field](const V& v) { return v.t->nerf_config().*field; },
	               [field](V& v, T x) {
		               v.t->nerf_config().*field = x;
		               v.t->push_nerf_config();
	               });
}

}  // namespace

PYBIND11_MODULE(pyngp, m) {
	m.doc() = "instant-ngp Testbed on MI355X (gfx950): the reference's pyngp surface over the engine's C-ABI";
	g_module_file = m.attr("__file__").cast<std::string>();

	py::enum_<ETestbedMode>(m, "TestbedMode")
		.value("Nerf", ETestbedMode::Nerf).value("Sdf", ETestbedMode::Sdf).value("Image", ETestbedMode::Image)
		.value("Volume", ETestbedMode::Volume).value("None", ETestbedMode::None).export_values();
	m.def("mode_from_scene", &mode_from_scene);
	m.def("mode_from_string", &mode_from_string);
	py::enum_<ERenderMode>(m, "RenderMode")
		.value("AO", ERenderMode::AO).value("Shade", ERenderMode::Shade).value("Normals", ERenderMode::Normals)
		.value("Positions", ERenderMode::Positions).value("Depth", ERenderMode::Depth).value("Distortion", ERenderMode::Distortion)
		.value("Cost", ERenderMode::Cost).value("Slice", ERenderMode::Slice).export_values();
	py::enum_<ELossType>(m, "LossType")
		.value("L2", ELossType::L2).value("L1", ELossType::L1).value("Mape", ELossType::Mape).value("Smape", ELossType::Smape)
		.value("Huber", ELossType::Huber).value("SmoothL1", ELossType::Huber).value("LogL1", ELossType::LogL1)
		.value("RelativeL2", ELossType::RelativeL2);
	py::enum_<ENerfActivation>(m, "NerfActivation")
		.value("None", ENerfActivation::None).value("ReLU", ENerfActivation::ReLU).value("Logistic", ENerfActivation::Logistic)
		.value("Exponential", ENerfActivation::Exponential);
	py::enum_<ERandomMode>(m, "RandomMode").value("Random", ERandomMode::Random).value("Stratified", ERandomMode::Stratified);

	py::class_<Testbed> testbed(m, "Testbed");
	testbed
		.def(py::init<ETestbedMode>(), py::arg("mode") = ETestbedMode::None)
		.def(py::init([](ETestbedMode mode, const std::string& data_path, const std::string& network_config_path) {
			     auto t = std::make_unique<Testbed>(mode);
			     if (!data_path.empty()) load_training_data(*t, data_path);
			     if (!network_config_path.empty()) t->reload_network_from_file(network_config_path);
			     return t;
		     }),
		     py::arg("mode"), py::arg("data_path"), py::arg("network_config_path"))
		.def_property_readonly("mode", &Testbed::mode)
		.def("load_training_data", &load_training_data, "Load training data from a given path.")
		.def("clear_training_data", &Testbed::clear_training_data, "Clears training data to free up GPU memory.")
		.def("frame", &Testbed::frame, py::call_guard<py::gil_scoped_release>(),
		     "Process a single frame (headless: one training step when shall_train).")
		.def("train", &Testbed::train, py::call_guard<py::gil_scoped_release>(), py::arg("batch_size"),
		     "Perform a single training step with a specified batch size.")
		.def("reset", &Testbed::reset_network, py::arg("reset_density_grid") = true, "Reset training.")
		.def("reload_network_from_file", &Testbed::reload_network_from_file, py::arg("path") = "",
		     "Reload the network from a config file.")
		.def("reload_network_from_json",
		     [](Testbed& t, py::object json, const std::string&) {
			     t.reload_network_from_json(py::module_::import("json").attr("dumps")(json).cast<std::string>());
		     },
		     py::arg("json"), py::arg("config_base_path") = "", "Reload the network from a json object.")
		.def("n_params", &Testbed::n_params, "Number of trainable parameters")
		.def("n_encoding_params", &Testbed::n_encoding_params, "Number of trainable parameters in the encoding")
		.def("save_snapshot", &Testbed::save_snapshot, py::arg("path"), py::arg("include_optimizer_state") = false,
		     py::arg("compress") = true, py::call_guard<py::gil_scoped_release>(),
		     "Save a snapshot of the currently trained model (.ingp: gzip'd msgpack).")
		.def("load_snapshot", &Testbed::load_snapshot, py::arg("path"), py::call_guard<py::gil_scoped_release>(),
		     "Load a previously saved snapshot")
		.def("load_file", &load_file, py::arg("path"),
		     "Load a file and automatically determine how to handle it: a snapshot, a network config or training data.")
		.def("render",
		     [](Testbed& t, uint32_t width, uint32_t height, uint32_t spp, bool linear, float, float, float, float) {
			     std::vector<float> img;
			     {
				     py::gil_scoped_release nogil;
				     img = t.render(width, height, spp, linear);
			     }
			     py::array_t<float> a({(py::ssize_t)height, (py::ssize_t)width, (py::ssize_t)4});
			     std::memcpy(a.mutable_data(), img.data(), img.size() * sizeof(float));
			     return a;
		     },
		     py::arg("width") = 1920, py::arg("height") = 1080, py::arg("spp") = 1, py::arg("linear") = true,
		     py::arg("start_t") = -1.f, py::arg("end_t") = -1.f, py::arg("fps") = 30.f, py::arg("shutter_fraction") = 1.0f,
		     "Renders an image at the requested resolution. Does not require a window.")
		.def_readwrite("shall_train", &Testbed::m_train)
		.def_readwrite("training_batch_size", &Testbed::m_training_batch_size)
		.def_readwrite("render_mode", &Testbed::m_render_mode)
		.def_readwrite("fov_axis", &Testbed::m_fov_axis)
		.def_readwrite("zoom", &Testbed::m_zoom)
		.def_property(
			"background_color", [](const Testbed& t) { return std::vector<float>(t.m_background_color, t.m_background_color + 4); },
			[](Testbed& t, const std::vector<float>& c) {
				if (c.size() != 4) throw std::runtime_error("background_color: 4 values (RGBA, linear)");
				std::copy(c.begin(), c.end(), t.m_background_color);
			})
		// m_camera: mat4x3 (columns = the camera's x, y, z axes and its position), as a [3 x 4] array
		.def_property(
			"camera_matrix",
			[](const Testbed& t) {
				py::array_t<float> a({3, 4});
				auto r = a.mutable_unchecked<2>();
				for (int c = 0; c < 4; ++c)
					for (int k = 0; k < 3; ++k) r(k, c) = t.m_camera[c * 3 + k];
				return a;
			},
			[](Testbed& t, py::array_t<float, py::array::c_style | py::array::forcecast> a) {
				if (a.ndim() != 2 || a.shape(0) != 3 || a.shape(1) != 4) throw std::runtime_error("camera_matrix: a [3 x 4] array");
				auto r = a.unchecked<2>();
				for (int c = 0; c < 4; ++c)
					for (int k = 0; k < 3; ++k) t.m_camera[c * 3 + k] = r(k, c);
			})
		.def("set_camera_to_training_view", &Testbed::set_camera_to_training_view, py::arg("view"))
		.def("first_training_view", [](Testbed& t) { t.set_camera_to_training_view(0); })
		.def("last_training_view", [](Testbed& t) { t.set_camera_to_training_view(t.n_training_views() - 1); })
		.def("previous_training_view",
		     [](Testbed& t) { t.set_camera_to_training_view(t.m_training_view == 0 ? t.n_training_views() - 1 : t.m_training_view - 1); })
		.def("next_training_view", [](Testbed& t) { t.set_camera_to_training_view((t.m_training_view + 1) % t.n_training_views()); })
		.def_property_readonly("loss", &Testbed::loss)
		.def_property_readonly("training_step", &Testbed::training_step)
		.def_readonly("bounding_radius", &Testbed::m_bounding_radius)
		.def_property_readonly("nerf", py::cpp_function([](Testbed& t) { return NerfView{&t}; }, py::keep_alive<0, 1>()))
		.def_property_readonly("sdf", py::cpp_function([](Testbed& t) { return SdfView{&t}; }, py::keep_alive<0, 1>()))
		.def_property_readonly("image", py::cpp_function([](Testbed& t) { return ImageView{&t}; }, py::keep_alive<0, 1>()));

	py::class_<NerfView> nerf(testbed, "Nerf");
	nerf.def_property_readonly("training", py::cpp_function([](NerfView& v) { return NerfTrainingView{v.t}; }, py::keep_alive<0, 1>()))
		.def_property("rgb_activation", [](NerfView& v) { return (ENerfActivation)v.t->nerf_config().rgb_activation; },
		              [](NerfView& v, ENerfActivation a) { v.t->nerf_config().rgb_activation = (uint32_t)a; v.t->push_nerf_config(); })
		.def_property("density_activation", [](NerfView& v) { return (ENerfActivation)v.t->nerf_config().density_activation; },
		              [](NerfView& v, ENerfActivation a) { v.t->nerf_config().density_activation = (uint32_t)a; v.t->push_nerf_config(); })
		.def_property("render_min_transmittance", [](NerfView& v) { return v.t->m_render_min_transmittance; },
		              [](NerfView& v, float x) { v.t->m_render_min_transmittance = x; })
		.def_property("rendering_min_transmittance", [](NerfView& v) { return v.t->m_render_min_transmittance; },
		              [](NerfView& v, float x) { v.t->m_render_min_transmittance = x; })
		.def_property("render_with_lens_distortion", [](NerfView& v) { return v.t->m_render_with_lens_distortion; },
		              [](NerfView& v, bool x) { v.t->m_render_with_lens_distortion = x; });
	nerf_knob(nerf, "cone_angle_constant", &ngp_nerf_config::cone_angle_constant);

	py::class_<NerfTrainingView> ntr(nerf, "Training");
	nerf_knob(ntr, "random_bg_color", &ngp_nerf_config::random_bg_color);
	nerf_knob(ntr, "linear_colors", &ngp_nerf_config::linear_colors);
	nerf_knob(ntr, "snap_to_pixel_centers", &ngp_nerf_config::snap_to_pixel_centers);
	nerf_knob(ntr, "near_distance", &ngp_nerf_config::near_distance);
	ntr.def_property("loss_type", [](NerfTrainingView& v) { return (ELossType)v.t->nerf_config().loss_type; },
	                 [](NerfTrainingView& v, ELossType l) { v.t->nerf_config().loss_type = (uint32_t)l; v.t->push_nerf_config(); })
		.def_property_readonly("n_images_for_training", [](NerfTrainingView& v) { return v.t->n_training_views(); })
		.def_property_readonly("dataset", py::cpp_function([](NerfTrainingView& v) { return NerfDatasetView{v.t}; }, py::keep_alive<0, 1>()));

	py::class_<NerfDatasetView>(m, "NerfDataset")
		.def_property_readonly("n_images", [](NerfDatasetView& v) { return v.t->n_training_views(); })
		.def_property_readonly("aabb_scale", [](NerfDatasetView& v) { return v.t->aabb_scale(); })
		.def_property_readonly("metadata", [](NerfDatasetView& v) {
			py::list out;
			for (const ngp_nerf_image& im : v.t->nerf_images()) {
				py::dict d;
				d["resolution"] = std::vector<uint32_t>{im.width, im.height};
				d["focal_length"] = std::vector<float>{im.focal_length[0], im.focal_length[1]};
				d["principal_point"] = std::vector<float>{im.principal_point[0], im.principal_point[1]};
				d["lens"] = py::make_tuple(im.lens_mode, std::vector<float>(im.lens_params, im.lens_params + 4));
				out.append(d);
			}
			return out;
		})
		.def_property_readonly("transforms", [](NerfDatasetView& v) {
			py::list out;
			for (const ngp_nerf_image& im : v.t->nerf_images()) {
				py::array_t<float> a({3, 4});
				auto r = a.mutable_unchecked<2>();
				for (int c = 0; c < 4; ++c)
					for (int k = 0; k < 3; ++k) r(k, c) = im.xform[c * 3 + k];
				out.append(a);
			}
			return out;
		});

	py::class_<SdfView> sdf(testbed, "Sdf");
	sdf.def_property_readonly("training", py::cpp_function([](SdfView& v) { return SdfTrainingView{v.t}; }, py::keep_alive<0, 1>()));
	py::class_<SdfTrainingView>(sdf, "Training")
		.def_property("generate_sdf_data_online", [](SdfTrainingView& v) { return v.t->m_sdf_generate_online; },
		              [](SdfTrainingView& v, bool x) { v.t->m_sdf_generate_online = x; })
		.def_property("surface_offset_scale", [](SdfTrainingView& v) { return v.t->m_sdf_surface_offset_scale; },
		              [](SdfTrainingView& v, float x) { v.t->m_sdf_surface_offset_scale = x; });

	py::class_<ImageView> image(testbed, "Image");
	image.def_property_readonly("training", py::cpp_function([](ImageView& v) { return ImageTrainingView{v.t}; }, py::keep_alive<0, 1>()))
		.def_property("random_mode", [](ImageView& v) { return (ERandomMode)v.t->image_config().random_mode; },
		              [](ImageView& v, ERandomMode r) { v.t->image_config().random_mode = (uint32_t)r; });
	py::class_<ImageTrainingView>(image, "Training")
		.def_property("snap_to_pixel_centers", [](ImageTrainingView& v) { return (bool)v.t->image_config().snap_to_pixel_centers; },
		              [](ImageTrainingView& v, bool x) { v.t->image_config().snap_to_pixel_centers = x; })
		.def_property("linear_colors", [](ImageTrainingView& v) { return (bool)v.t->image_config().linear_colors; },
		              [](ImageTrainingView& v, bool x) { v.t->image_config().linear_colors = x; });

	// engine extension for tests and tools: the network config in use (JSON text) and the default of a mode
	m.def("default_network_config", [](ETestbedMode mode) { return default_network_config(mode); });
	testbed.def_property_readonly("network_config", &Testbed::network_config);
}
