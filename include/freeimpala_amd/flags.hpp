// flags.hpp -- a small strict command-line parser with the chained registration style of the
// argparse library the reference's binaries use (reference cmd/freeimpala/main.cpp:38-121:
// add_argument(short, long).help(..).default_value(..).scan<'i', int>(); parse_args throws
// std::runtime_error on an unknown flag or a malformed value, :131-137; get<T>(name)).
// The learner flags are registered by freeimpala_amd::add_learner_arguments(parser), a template
// that works on this parser and on argparse::ArgumentParser alike, so a binary that parses
// strictly accepts --seq-length & co. (tools/fi_freeimpala.cpp).
#pragma once

#include <cerrno>
#include <cstdlib>
#include <deque>
#include <initializer_list>
#include <ostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

namespace freeimpala_amd {

class ArgumentParser {
public:
    class Argument {
    public:
        Argument& help(std::string h) {
            help_ = std::move(h);
            return *this;
        }
        template <class T>
        Argument& default_value(T v) {
            if constexpr (std::is_same_v<std::decay_t<T>, std::string> || std::is_same_v<std::decay_t<T>, const char*> ||
                          std::is_array_v<std::remove_reference_t<T>>) {
                default_ = std::string(v);
            } else {
                default_ = std::to_string(v);
                if (kind_ == 's') kind_ = std::is_floating_point_v<T> ? 'g' : (std::is_unsigned_v<T> ? 'u' : 'i');
            }
            has_default_ = true;
            return *this;
        }
        template <char K, class T>
        Argument& scan() {
            kind_ = K == 'g' || K == 'f' ? 'g' : K;
            return *this;
        }
        template <class... S>
        Argument& choices(S&&... s) {
            (choices_.push_back(std::string(s)), ...);
            return *this;
        }

    private:
        friend class ArgumentParser;
        std::vector<std::string> names_;
        std::string help_, default_, value_;
        std::vector<std::string> choices_;
        char kind_ = 's';  // s string, i int, u unsigned, g floating
        bool has_default_ = false, used_ = false;
    };

    explicit ArgumentParser(std::string prog = "") : prog_(std::move(prog)) {}

    void add_description(std::string d) { desc_ = std::move(d); }

    template <class... N>
    Argument& add_argument(N&&... names) {
        args_.emplace_back();
        (args_.back().names_.push_back(std::string(names)), ...);
        for (const auto& n : args_.back().names_)
            for (size_t i = 0; i + 1 < args_.size(); ++i)
                for (const auto& m : args_[i].names_)
                    if (m == n) throw std::logic_error("flag registered twice: " + n);
        return args_.back();
    }

    // strict: every token must be a registered flag followed by its value ("--flag v" or
    // "--flag=v"); -h/--help throws with the usage text
    void parse_args(int argc, const char* const* argv) {
        for (int i = 1; i < argc; ++i) {
            std::string tok = argv[i], val;
            bool inline_val = false;
            if (tok == "-h" || tok == "--help") throw std::runtime_error(usage());
            const size_t eq = tok.find('=');
            if (tok.rfind("--", 0) == 0 && eq != std::string::npos) {
                val = tok.substr(eq + 1);
                tok = tok.substr(0, eq);
                inline_val = true;
            }
            Argument* a = find(tok);
            if (!a) throw std::runtime_error("Unknown argument: " + tok);
            if (!inline_val) {
                if (i + 1 >= argc) throw std::runtime_error(tok + ": expected a value");
                val = argv[++i];
            }
            check(*a, tok, val);
            a->value_ = val;
            a->used_ = true;
        }
    }

    template <class T>
    T get(const std::string& name) const {
        const Argument* a = find(name);
        if (!a) throw std::logic_error("No such argument: " + name);
        const std::string& s = a->used_ ? a->value_ : a->default_;
        if (!a->used_ && !a->has_default_) throw std::logic_error("No value provided for " + name);
        if constexpr (std::is_same_v<T, std::string>) {
            return s;
        } else if constexpr (std::is_floating_point_v<T>) {
            return (T)std::strtod(s.c_str(), nullptr);
        } else if constexpr (std::is_unsigned_v<T>) {
            return (T)std::strtoull(s.c_str(), nullptr, 10);
        } else {
            return (T)std::strtoll(s.c_str(), nullptr, 10);
        }
    }

    bool is_used(const std::string& name) const {
        const Argument* a = find(name);
        return a && a->used_;
    }

    std::string usage() const {
        std::ostringstream o;
        o << "Usage: " << prog_ << " [options]\n";
        if (!desc_.empty()) o << desc_ << "\n";
        for (const auto& a : args_) {
            o << "  ";
            for (size_t i = 0; i < a.names_.size(); ++i) o << (i ? ", " : "") << a.names_[i];
            o << "\t" << a.help_;
            if (a.has_default_) o << " [default: " << a.default_ << "]";
            o << "\n";
        }
        return o.str();
    }
    friend std::ostream& operator<<(std::ostream& os, const ArgumentParser& p) { return os << p.usage(); }

private:
    Argument* find(const std::string& n) {
        for (auto& a : args_)
            for (const auto& m : a.names_)
                if (m == n) return &a;
        return nullptr;
    }
    const Argument* find(const std::string& n) const { return const_cast<ArgumentParser*>(this)->find(n); }

    static void check(const Argument& a, const std::string& flag, const std::string& v) {
        if (!a.choices_.empty()) {
            bool ok = false;
            for (const auto& c : a.choices_) ok = ok || c == v;
            if (!ok) throw std::runtime_error("Invalid value for " + flag + ": " + v);
        }
        if (a.kind_ == 's') return;
        char* end = nullptr;
        errno = 0;
        if (a.kind_ == 'g') std::strtod(v.c_str(), &end);
        else if (a.kind_ == 'u') {
            if (!v.empty() && v[0] == '-') throw std::runtime_error("Invalid value for " + flag + ": " + v);
            std::strtoull(v.c_str(), &end, 10);
        } else std::strtoll(v.c_str(), &end, 10);
        if (v.empty() || *end || errno) throw std::runtime_error("Invalid value for " + flag + ": " + v);
    }

    std::string prog_, desc_;
    std::deque<Argument> args_;  // deque: an Argument& stays valid across later add_argument calls
};

}  // namespace freeimpala_amd
