// msgpack.h — MessagePack values for the .ingp snapshot format (host only).
//
// The reference writes its snapshot as nlohmann::json::to_msgpack of the network config with a
// "snapshot" member (src/testbed.cu:4873-4937), GPU buffers as msgpack binaries
// (tcnn gpu_memory_to_json_binary). This is the subset that format uses: nil, bool, integers,
// float32/64, str, bin, array, map (string keys, insertion order kept). Encoder picks the smallest
// encoding like nlohmann does; the decoder accepts every width.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "json.h"

namespace ngp {
namespace mp {

struct Value {
	enum Type { Nil, Bool, Int, UInt, Float, Str, Bin, Array, Map } type = Nil;
	bool b = false;
	int64_t i = 0;
	uint64_t u = 0;
	double f = 0;
	std::string s;                 // Str; Bin bytes
	std::vector<Value> arr;
	std::vector<std::pair<std::string, Value>> map;

	static Value nil() { return Value{}; }
	static Value boolean(bool v) { Value x; x.type = Bool; x.b = v; return x; }
	static Value uint(uint64_t v) { Value x; x.type = UInt; x.u = v; return x; }
	static Value sint(int64_t v) { if (v >= 0) return uint((uint64_t)v); Value x; x.type = Int; x.i = v; return x; }
	static Value real(double v) { Value x; x.type = Float; x.f = v; return x; }
	static Value str(std::string v) { Value x; x.type = Str; x.s = std::move(v); return x; }
	static Value bin(const void* p, size_t n) { Value x; x.type = Bin; x.s.assign((const char*)p, n); return x; }
	static Value array() { Value x; x.type = Array; return x; }
	static Value object() { Value x; x.type = Map; return x; }

	bool is_map() const { return type == Map; }
	const Value* find(const std::string& k) const {
		if (type != Map) return nullptr;
		for (auto& kv : map) if (kv.first == k) return &kv.second;
		return nullptr;
	}
	const Value& at(const std::string& k) const {
		const Value* v = find(k);
		if (!v) throw std::runtime_error("snapshot: missing key '" + k + "'");
		return *v;
	}
	Value& operator[](const std::string& k) {  // insert-or-get (Map)
		if (type == Nil) type = Map;
		if (type != Map) throw std::runtime_error("msgpack: not a map");
		for (auto& kv : map) if (kv.first == k) return kv.second;
		map.emplace_back(k, Value{});
		return map.back().second;
	}
	void erase(const std::string& k) {
		for (size_t j = 0; j < map.size(); ++j) if (map[j].first == k) { map.erase(map.begin() + j); return; }
	}
	double number() const {
		switch (type) {
			case Int: return (double)i;
			case UInt: return (double)u;
			case Float: return f;
			case Bool: return b ? 1.0 : 0.0;
			default: throw std::runtime_error("snapshot: expected a number");
		}
	}
	double number_or(const std::string& k, double d) const { const Value* v = find(k); return v ? v->number() : d; }
};

// ---- encoder --------------------------------------------------------------------------------
inline void put_be(std::string& o, uint64_t v, int bytes) {
	for (int k = bytes - 1; k >= 0; --k) o.push_back((char)((v >> (8 * k)) & 0xff));
}
inline void encode(const Value& v, std::string& o) {
	switch (v.type) {
		case Value::Nil: o.push_back((char)0xc0); return;
		case Value::Bool: o.push_back((char)(v.b ? 0xc3 : 0xc2)); return;
		case Value::UInt:
			if (v.u < 128) o.push_back((char)v.u);
			else if (v.u <= 0xff) { o.push_back((char)0xcc); put_be(o, v.u, 1); }
			else if (v.u <= 0xffff) { o.push_back((char)0xcd); put_be(o, v.u, 2); }
			else if (v.u <= 0xffffffffull) { o.push_back((char)0xce); put_be(o, v.u, 4); }
			else { o.push_back((char)0xcf); put_be(o, v.u, 8); }
			return;
		case Value::Int:
			if (v.i >= -32) o.push_back((char)(int8_t)v.i);
			else if (v.i >= INT8_MIN) { o.push_back((char)0xd0); put_be(o, (uint8_t)(int8_t)v.i, 1); }
			else if (v.i >= INT16_MIN) { o.push_back((char)0xd1); put_be(o, (uint16_t)(int16_t)v.i, 2); }
			else if (v.i >= INT32_MIN) { o.push_back((char)0xd2); put_be(o, (uint32_t)(int32_t)v.i, 4); }
			else { o.push_back((char)0xd3); put_be(o, (uint64_t)v.i, 8); }
			return;
		case Value::Float: {
			const float f32 = (float)v.f;
			if ((double)f32 == v.f || std::isnan(v.f)) {  // lossless as float32 (nlohmann write_compact_float)
				uint32_t bits;
				memcpy(&bits, &f32, 4);
				o.push_back((char)0xca);
				put_be(o, bits, 4);
			} else {
				uint64_t bits;
				memcpy(&bits, &v.f, 8);
				o.push_back((char)0xcb);
				put_be(o, bits, 8);
			}
			return;
		}
		case Value::Str: {
			const size_t n = v.s.size();
			if (n < 32) o.push_back((char)(0xa0 | n));
			else if (n <= 0xff) { o.push_back((char)0xd9); put_be(o, n, 1); }
			else if (n <= 0xffff) { o.push_back((char)0xda); put_be(o, n, 2); }
			else { o.push_back((char)0xdb); put_be(o, n, 4); }
			o += v.s;
			return;
		}
		case Value::Bin: {
			const size_t n = v.s.size();
			if (n <= 0xff) { o.push_back((char)0xc4); put_be(o, n, 1); }
			else if (n <= 0xffff) { o.push_back((char)0xc5); put_be(o, n, 2); }
			else { o.push_back((char)0xc6); put_be(o, n, 4); }
			o += v.s;
			return;
		}
		case Value::Array: {
			const size_t n = v.arr.size();
			if (n < 16) o.push_back((char)(0x90 | n));
			else if (n <= 0xffff) { o.push_back((char)0xdc); put_be(o, n, 2); }
			else { o.push_back((char)0xdd); put_be(o, n, 4); }
			for (auto& e : v.arr) encode(e, o);
			return;
		}
		case Value::Map: {
			const size_t n = v.map.size();
			if (n < 16) o.push_back((char)(0x80 | n));
			else if (n <= 0xffff) { o.push_back((char)0xde); put_be(o, n, 2); }
			else { o.push_back((char)0xdf); put_be(o, n, 4); }
			for (auto& kv : v.map) { encode(Value::str(kv.first), o); encode(kv.second, o); }
			return;
		}
	}
}

// ---- decoder --------------------------------------------------------------------------------
struct Reader {
	const uint8_t* p;
	size_t n, i = 0;
	uint64_t be(int bytes) {
		if (i + bytes > n) throw std::runtime_error("msgpack: truncated");
		uint64_t v = 0;
		for (int k = 0; k < bytes; ++k) v = (v << 8) | p[i++];
		return v;
	}
	std::string raw(size_t len) {
		if (i + len > n) throw std::runtime_error("msgpack: truncated");
		std::string s((const char*)p + i, len);
		i += len;
		return s;
	}
	Value value(int depth = 0) {
		if (depth > 64) throw std::runtime_error("msgpack: nesting too deep");
		const uint8_t c = (uint8_t)be(1);
		if (c <= 0x7f) return Value::uint(c);
		if (c >= 0xe0) return Value::sint((int8_t)c);
		if ((c & 0xe0) == 0xa0) return Value::str(raw(c & 0x1f));
		if ((c & 0xf0) == 0x90) return array(c & 0x0f, depth);
		if ((c & 0xf0) == 0x80) return object(c & 0x0f, depth);
		switch (c) {
			case 0xc0: return Value::nil();
			case 0xc2: return Value::boolean(false);
			case 0xc3: return Value::boolean(true);
			case 0xc4: { size_t l = be(1); Value v; v.type = Value::Bin; v.s = raw(l); return v; }
			case 0xc5: { size_t l = be(2); Value v; v.type = Value::Bin; v.s = raw(l); return v; }
			case 0xc6: { size_t l = be(4); Value v; v.type = Value::Bin; v.s = raw(l); return v; }
			case 0xca: { uint32_t b = (uint32_t)be(4); float f; memcpy(&f, &b, 4); return Value::real(f); }
			case 0xcb: { uint64_t b = be(8); double d; memcpy(&d, &b, 8); return Value::real(d); }
			case 0xcc: return Value::uint(be(1));
			case 0xcd: return Value::uint(be(2));
			case 0xce: return Value::uint(be(4));
			case 0xcf: return Value::uint(be(8));
			case 0xd0: return Value::sint((int8_t)be(1));
			case 0xd1: return Value::sint((int16_t)be(2));
			case 0xd2: return Value::sint((int32_t)be(4));
			case 0xd3: return Value::sint((int64_t)be(8));
			case 0xd9: return Value::str(raw(be(1)));
			case 0xda: return Value::str(raw(be(2)));
			case 0xdb: return Value::str(raw(be(4)));
			case 0xdc: return array(be(2), depth);
			case 0xdd: return array(be(4), depth);
			case 0xde: return object(be(2), depth);
			case 0xdf: return object(be(4), depth);
			// ext types (nlohmann writes binaries with a subtype as ext): keep the payload as Bin
			case 0xd4: case 0xd5: case 0xd6: case 0xd7: case 0xd8: {
				const size_t l = (size_t)1 << (c - 0xd4);
				be(1);
				Value v; v.type = Value::Bin; v.s = raw(l); return v;
			}
			case 0xc7: case 0xc8: case 0xc9: {
				const size_t l = be(c == 0xc7 ? 1 : c == 0xc8 ? 2 : 4);
				be(1);
				Value v; v.type = Value::Bin; v.s = raw(l); return v;
			}
		}
		throw std::runtime_error("msgpack: unsupported type byte");
	}
	Value array(size_t len, int depth) {
		Value v = Value::array();
		for (size_t k = 0; k < len; ++k) v.arr.push_back(value(depth + 1));
		return v;
	}
	Value object(size_t len, int depth) {
		Value v = Value::object();
		for (size_t k = 0; k < len; ++k) {
			Value key = value(depth + 1);
			if (key.type != Value::Str) throw std::runtime_error("msgpack: map key must be a string");
			v.map.emplace_back(key.s, value(depth + 1));
		}
		return v;
	}
};

inline Value decode(const std::string& bytes) {
	Reader r{(const uint8_t*)bytes.data(), bytes.size()};
	Value v = r.value();
	return v;
}

// ---- JSON bridges -----------------------------------------------------------------------------
inline Value from_json(const Json& j) {
	switch (j.type) {
		case Json::Null: return Value::nil();
		case Json::Bool: return Value::boolean(j.b);
		case Json::Number:
			if (std::floor(j.num) == j.num && std::fabs(j.num) < 9.0e15) return Value::sint((int64_t)j.num);
			return Value::real(j.num);
		case Json::String: return Value::str(j.str);
		case Json::Array: { Value v = Value::array(); for (auto& e : j.arr) v.arr.push_back(from_json(e)); return v; }
		case Json::Object: { Value v = Value::object(); for (auto& kv : j.obj) v.map.emplace_back(kv.first, from_json(kv.second)); return v; }
	}
	return Value::nil();
}

inline void json_escape(const std::string& s, std::string& o) {
	o.push_back('"');
	for (char c : s) {
		if (c == '"' || c == '\\') { o.push_back('\\'); o.push_back(c); }
		else if (c == '\n') o += "\\n";
		else if (c == '\t') o += "\\t";
		else o.push_back(c);
	}
	o.push_back('"');
}
// JSON text of a value; binaries are written as their byte count ({"binary_bytes": n})
inline void to_json_text(const Value& v, std::string& o) {
	char buf[64];
	switch (v.type) {
		case Value::Nil: o += "null"; return;
		case Value::Bool: o += v.b ? "true" : "false"; return;
		case Value::Int: snprintf(buf, sizeof buf, "%lld", (long long)v.i); o += buf; return;
		case Value::UInt: snprintf(buf, sizeof buf, "%llu", (unsigned long long)v.u); o += buf; return;
		case Value::Float: snprintf(buf, sizeof buf, "%.17g", v.f); o += buf; return;
		case Value::Str: json_escape(v.s, o); return;
		case Value::Bin: snprintf(buf, sizeof buf, "{\"binary_bytes\": %zu}", v.s.size()); o += buf; return;
		case Value::Array:
			o.push_back('[');
			for (size_t k = 0; k < v.arr.size(); ++k) { if (k) o += ", "; to_json_text(v.arr[k], o); }
			o.push_back(']');
			return;
		case Value::Map:
			o.push_back('{');
			for (size_t k = 0; k < v.map.size(); ++k) {
				if (k) o += ", ";
				json_escape(v.map[k].first, o);
				o += ": ";
				to_json_text(v.map[k].second, o);
			}
			o.push_back('}');
			return;
	}
}

}  // namespace mp
}  // namespace ngp
