// options.hpp — command line of the BSMR-sddmm drop-in binary.
// Same flags, defaults and parsing behaviour as the reference Options (include/Options.hpp:13-124):
// -f/-F file, -k/-K K, -a/-A alpha, -d/-D delta, -t/-T test mode, -l/-L log directory; every flag
// takes a value; duplicates are warned about and skipped; parse errors are printed and ignored;
// with no '-' flags the positional form "prog file K" applies.
#pragma once

#include <iostream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace cli {

inline std::string parent_folder(const std::string& path) {
    if (path.empty()) return "";
    const size_t pos = path.find_last_of("/\\");
    if (pos == std::string::npos) std::cerr << "Warning. The input path has no parent folder" << std::endl;
    return pos == std::string::npos ? "" : path.substr(0, pos + 1);
}

inline std::string file_name(const std::string& path) {
    if (path.empty()) return "";
    const size_t pos = path.find_last_of("/\\");
    if (pos == std::string::npos) std::cerr << "Warning. The input path has no parent folder" << std::endl;
    return pos == std::string::npos ? path : path.substr(pos + 1);
}

class Options {
public:
    Options(int argc, const char* const argv[]) {
        programPath_ = parent_folder(argv[0]);
        programName_ = file_name(argv[0]);
        std::vector<int> idx;
        for (int i = 1; i < argc; ++i)
            if (argv[i][0] == '-') idx.push_back(i);
        std::unordered_map<std::string, std::string> kv;  // same container => same parse order
        for (int i : idx) {
            const std::string opt = argv[i];
            if (kv.find(opt) != kv.end()) {
                std::cerr << "Option " << opt << "is duplicated." << std::endl;
                continue;
            }
            if (i + 1 >= argc) {
                std::cerr << "Option " << opt << "requires an argument." << std::endl;
                continue;
            }
            kv[opt] = argv[i + 1];
        }
        for (const auto& p : kv) parse(p.first, p.second);
        if (kv.empty() && argc > 1) {
            inputFile_ = argv[1];
            if (argc > 2) {
                K_ = std::stoi(argv[2]);
            } else {
                // the reference reads argv[2] out of bounds here; we keep the default K
                std::cerr << "Missing K argument; using K = " << K_ << std::endl;
            }
        }
    }

    std::string inputFile() const { return inputFile_; }
    size_t K() const { return K_; }
    int numIterations() const { return numIterations_; }
    float alpha() const { return alpha_; }
    float delta() const { return delta_; }
    bool testMode() const { return testMode_; }
    std::string outputLogDirectory() const { return logDir_; }

private:
    std::string programPath_, programName_, inputFile_, logDir_;
    size_t K_ = 32;
    int numIterations_ = 10;
    float alpha_ = 0.3f;
    float delta_ = 0.3f;
    bool testMode_ = false;

    void parse(const std::string& o, const std::string& v) {
        try {
            if (o == "-F" || o == "-f") inputFile_ = v;
            if (o == "-K" || o == "-k") K_ = std::stoi(v);
            if (o == "-A" || o == "-a") alpha_ = std::stof(v);
            if (o == "-D" || o == "-d") delta_ = std::stof(v);
            if (o == "-t" || o == "-T") testMode_ = std::stoi(v);
            if (o == "-l" || o == "-L") logDir_ = v;
        } catch (const std::invalid_argument& e) {
            std::cerr << "Invalid argument: " << e.what() << std::endl;
        } catch (const std::out_of_range& e) {
            std::cerr << "Out of range: " << e.what() << std::endl;
        }
    }
};

}  // namespace cli
