// A small JSON reader for the operator modules' configuration strings (the tcnn-shaped C-ABI takes the
// encoding / network objects of configs/nerf/*.json as text, as tcnn::cpp::create_* take nlohmann::json).
// Objects, arrays, numbers, strings, true / false / null; // and /* */ comments are skipped like the
// reference's config loader (testbed.cu:73-91) does before parsing. Throws std::runtime_error on bad input.
#pragma once
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace neus {

struct JsonValue {
	enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
	bool b = false;
	double num = 0.0;
	std::string str;
	std::vector<JsonValue> arr;
	std::map<std::string, JsonValue> obj;

	bool has(const std::string& k) const { return kind == Object && obj.count(k) != 0; }
	const JsonValue& at(const std::string& k) const {
		auto it = obj.find(k);
		if (kind != Object || it == obj.end()) throw std::runtime_error("json: missing key '" + k + "'");
		return it->second;
	}
	double number(const std::string& k, double def) const {
		if (!has(k)) return def;
		const JsonValue& v = at(k);
		if (v.kind == Number) return v.num;
		if (v.kind == Bool) return v.b ? 1.0 : 0.0;
		throw std::runtime_error("json: '" + k + "' is not a number");
	}
	std::string string(const std::string& k, const std::string& def) const {
		if (!has(k)) return def;
		const JsonValue& v = at(k);
		if (v.kind != String) throw std::runtime_error("json: '" + k + "' is not a string");
		return v.str;
	}
	const JsonValue& object(const std::string& k) const {
		static const JsonValue empty = [] { JsonValue e; e.kind = Object; return e; }();
		if (!has(k)) return empty;
		const JsonValue& v = at(k);
		if (v.kind != Object) throw std::runtime_error("json: '" + k + "' is not an object");
		return v;
	}
};

class JsonParser {
public:
	explicit JsonParser(const std::string& text) : s_(text) {}
	JsonValue parse() {
		JsonValue v = value();
		ws();
		if (i_ != s_.size()) fail("trailing characters");
		return v;
	}

private:
	const std::string& s_;
	size_t i_ = 0;

	[[noreturn]] void fail(const char* what) const { throw std::runtime_error(std::string("json: ") + what + " at offset " + std::to_string(i_)); }
	void ws() {
		for (;;) {
			while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\t' || s_[i_] == '\n' || s_[i_] == '\r')) ++i_;
			if (i_ + 1 < s_.size() && s_[i_] == '/' && s_[i_ + 1] == '/') {
				while (i_ < s_.size() && s_[i_] != '\n') ++i_;
			} else if (i_ + 1 < s_.size() && s_[i_] == '/' && s_[i_ + 1] == '*') {
				const size_t e = s_.find("*/", i_ + 2);
				if (e == std::string::npos) fail("unterminated comment");
				i_ = e + 2;
			} else {
				return;
			}
		}
	}
	bool lit(const char* w) {
		const size_t n = std::char_traits<char>::length(w);
		if (s_.compare(i_, n, w) == 0) { i_ += n; return true; }
		return false;
	}
	std::string str() {
		if (s_[i_] != '"') fail("expected a string");
		++i_;
		std::string out;
		while (i_ < s_.size() && s_[i_] != '"') {
			char c = s_[i_++];
			if (c == '\\') {
				if (i_ >= s_.size()) fail("bad escape");
				const char e = s_[i_++];
				switch (e) {
				case 'n': out += '\n'; break;
				case 't': out += '\t'; break;
				case 'r': out += '\r'; break;
				case 'b': out += '\b'; break;
				case 'f': out += '\f'; break;
				case 'u': {  // code points below 0x80 only (config keys and values are ASCII)
					if (i_ + 4 > s_.size()) fail("bad \\u escape");
					const long cp = std::strtol(s_.substr(i_, 4).c_str(), nullptr, 16);
					out += cp < 0x80 ? (char)cp : '?';
					i_ += 4;
					break;
				}
				default: out += e;
				}
			} else {
				out += c;
			}
		}
		if (i_ >= s_.size()) fail("unterminated string");
		++i_;
		return out;
	}
	JsonValue value() {
		ws();
		if (i_ >= s_.size()) fail("unexpected end");
		JsonValue v;
		const char c = s_[i_];
		if (c == '{') {
			v.kind = JsonValue::Object;
			++i_;
			ws();
			if (i_ < s_.size() && s_[i_] == '}') { ++i_; return v; }
			for (;;) {
				ws();
				std::string k = str();
				ws();
				if (i_ >= s_.size() || s_[i_] != ':') fail("expected ':'");
				++i_;
				v.obj[k] = value();
				ws();
				if (i_ < s_.size() && s_[i_] == ',') { ++i_; continue; }
				if (i_ < s_.size() && s_[i_] == '}') { ++i_; return v; }
				fail("expected ',' or '}'");
			}
		}
		if (c == '[') {
			v.kind = JsonValue::Array;
			++i_;
			ws();
			if (i_ < s_.size() && s_[i_] == ']') { ++i_; return v; }
			for (;;) {
				v.arr.push_back(value());
				ws();
				if (i_ < s_.size() && s_[i_] == ',') { ++i_; continue; }
				if (i_ < s_.size() && s_[i_] == ']') { ++i_; return v; }
				fail("expected ',' or ']'");
			}
		}
		if (c == '"') { v.kind = JsonValue::String; v.str = str(); return v; }
		if (lit("true")) { v.kind = JsonValue::Bool; v.b = true; return v; }
		if (lit("false")) { v.kind = JsonValue::Bool; v.b = false; return v; }
		if (lit("null")) return v;
		char* end = nullptr;
		v.num = std::strtod(s_.c_str() + i_, &end);
		if (end == s_.c_str() + i_) fail("unexpected character");
		i_ = (size_t)(end - s_.c_str());
		v.kind = JsonValue::Number;
		return v;
	}
};

inline JsonValue parse_json(const std::string& text) { return JsonParser(text).parse(); }

}  // namespace neus
