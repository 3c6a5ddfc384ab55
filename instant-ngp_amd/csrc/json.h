// json.h — minimal JSON reader for network/encoding/optimizer configs (the reference's configs,
// e.g. configs/image/base.json, carry // comments, which are accepted).
#pragma once
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace ngp {

struct Json {
	enum Type { Null, Bool, Number, String, Array, Object } type = Null;
	bool b = false;
	double num = 0;
	std::string str;
	std::vector<Json> arr;
	std::map<std::string, Json> obj;

	bool contains(const std::string& k) const { return type == Object && obj.count(k); }
	const Json& operator[](const std::string& k) const {
		auto it = obj.find(k);
		if (type != Object || it == obj.end()) throw std::runtime_error("json: missing key '" + k + "'");
		return it->second;
	}
	double number_or(const std::string& k, double d) const { return contains(k) ? (*this)[k].num : d; }
	std::string string_or(const std::string& k, const std::string& d) const { return contains(k) ? (*this)[k].str : d; }

	// compact JSON text (numbers with enough digits to round-trip a double)
	std::string dump() const {
		switch (type) {
		case Null: return "null";
		case Bool: return b ? "true" : "false";
		case Number: {
			char buf[32];
			snprintf(buf, sizeof(buf), "%.17g", num);
			return buf;
		}
		case String: return quote(str);
		case Array: {
			std::string o = "[";
			for (size_t i = 0; i < arr.size(); ++i) o += (i ? "," : "") + arr[i].dump();
			return o + "]";
		}
		case Object: {
			std::string o = "{";
			bool first = true;
			for (const auto& kv : obj) {
				o += (first ? "" : ",") + quote(kv.first) + ":" + kv.second.dump();
				first = false;
			}
			return o + "}";
		}
		}
		return "null";
	}
	static std::string quote(const std::string& s) {
		std::string o = "\"";
		for (char c : s) {
			if (c == '"' || c == '\\') { o += '\\'; o += c; }
			else if (c == '\n') o += "\\n";
			else if (c == '\t') o += "\\t";
			else o += c;
		}
		return o + "\"";
	}

	static Json parse(const std::string& s) {
		size_t i = 0;
		Json j = parse_value(s, i);
		skip(s, i);
		if (i != s.size()) throw std::runtime_error("json: trailing characters");
		return j;
	}

private:
	static void skip(const std::string& s, size_t& i) {
		for (;;) {
			while (i < s.size() && isspace((unsigned char)s[i])) ++i;
			if (i + 1 < s.size() && s[i] == '/' && s[i + 1] == '/') {
				while (i < s.size() && s[i] != '\n') ++i;
			} else if (i + 1 < s.size() && s[i] == '/' && s[i + 1] == '*') {
				size_t e = s.find("*/", i + 2);
				i = e == std::string::npos ? s.size() : e + 2;
			} else break;
		}
	}
	static Json parse_value(const std::string& s, size_t& i) {
		skip(s, i);
		if (i >= s.size()) throw std::runtime_error("json: unexpected end");
		Json j;
		const char c = s[i];
		if (c == '{') {
			j.type = Object; ++i;
			skip(s, i);
			if (s[i] == '}') { ++i; return j; }
			for (;;) {
				skip(s, i);
				Json k = parse_value(s, i);
				if (k.type != String) throw std::runtime_error("json: object key must be a string");
				skip(s, i);
				if (s[i] != ':') throw std::runtime_error("json: expected ':'");
				++i;
				j.obj[k.str] = parse_value(s, i);
				skip(s, i);
				if (s[i] == ',') { ++i; skip(s, i); if (s[i] == '}') { ++i; return j; } continue; }
				if (s[i] == '}') { ++i; return j; }
				throw std::runtime_error("json: expected ',' or '}'");
			}
		}
		if (c == '[') {
			j.type = Array; ++i;
			skip(s, i);
			if (s[i] == ']') { ++i; return j; }
			for (;;) {
				j.arr.push_back(parse_value(s, i));
				skip(s, i);
				if (s[i] == ',') { ++i; skip(s, i); if (s[i] == ']') { ++i; return j; } continue; }
				if (s[i] == ']') { ++i; return j; }
				throw std::runtime_error("json: expected ',' or ']'");
			}
		}
		if (c == '"') {
			j.type = String; ++i;
			while (i < s.size() && s[i] != '"') {
				if (s[i] == '\\' && i + 1 < s.size()) {
					char e = s[i + 1];
					j.str += e == 'n' ? '\n' : e == 't' ? '\t' : e;
					i += 2;
				} else j.str += s[i++];
			}
			++i;
			return j;
		}
		if (s.compare(i, 4, "true") == 0) { j.type = Bool; j.b = true; i += 4; return j; }
		if (s.compare(i, 5, "false") == 0) { j.type = Bool; i += 5; return j; }
		if (s.compare(i, 4, "null") == 0) { i += 4; return j; }
		char* end = nullptr;
		j.num = strtod(s.c_str() + i, &end);
		if (end == s.c_str() + i) throw std::runtime_error("json: bad value");
		j.type = Number;
		i = end - s.c_str();
		return j;
	}
};

inline bool iequals(const std::string& a, const std::string& b) {
	if (a.size() != b.size()) return false;
	for (size_t i = 0; i < a.size(); ++i)
		if (tolower((unsigned char)a[i]) != tolower((unsigned char)b[i])) return false;
	return true;
}

}  // namespace ngp
