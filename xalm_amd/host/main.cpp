// main.cpp — `xalm` CLI: the reference's argument surface (jubruckne/Xalm src/main.cpp:381-549)
// over the MI355X decode path.
//
//   xalm <checkpoint.xalm> [-m completion|perplexity] [-d hip|cpu] [-i prompt | -f file]
//                          [-T context] [-n steps] [-g 0|1]
//
// -d selects the device as in the reference (src/main.cpp:465-477); this build ships the HIP
// device.  -g 1 runs the greedy loop on the device (no host round trip per token); -g 0
// (default) samples on the host each step exactly like run_completion (src/main.cpp:105-115).
// Stats are wall clock (the reference divides by user+sys CPU time, src/profiler.h:124-129).
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "xalm.h"

using namespace xalm;
using clk = std::chrono::steady_clock;

static void error_usage() {
    fprintf(stderr, "Usage:   xalm <checkpoint> [options]\n");
    fprintf(stderr, "Example: xalm model.xalm -i \"Q: What is the meaning of life?\"\n");
    fprintf(stderr, "Options:\n");
    fprintf(stderr, "  -h Display this help message\n");
    fprintf(stderr, "  -d [hip,cpu] which device to use (default - hip)\n");
    fprintf(stderr, "  -m [completion,perplexity] which mode to run in (default - completion)\n");
    fprintf(stderr, "  -T <int> sliding window context length (0 - max)\n");
    fprintf(stderr, "  -n <int> number of steps in completion mode, default 128. 0 = max_seq_len, -1 = infinite\n");
    fprintf(stderr, "  -g <0|1> greedy decode loop on the device (default 0)\n");
    fprintf(stderr, "  Choose one:\n");
    fprintf(stderr, "    -i <string> input prompt\n");
    fprintf(stderr, "    -f <filepath> input file with prompt\n");
    exit(1);
}

static double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

static void print_ids(const std::vector<int>& ids) {
    printf("tokens: [");
    for (size_t i = 0; i < ids.size(); i++) printf(i ? ",%d" : "%d", ids[i]);
    printf("]\n");
}

// run_completion, src/main.cpp:44-128
static void run_completion(const std::string& path, Device dev, const std::string& prompt, int context, int num_steps,
                           bool device_loop) {
    const XalmFile file = XalmFile::load(path);
    const Model model = Model::from_xalm(file, context, dev);
    InferenceState state(model.config);
    const Sampler sampler(model.config);
    const Tokenizer tokenizer(file);
    printf("Model active bytes(m): %zu\n", model.active_bytes(model.config.max_seq_len) / (1024 * 1024));
    if (num_steps == 0) num_steps = model.config.max_seq_len;
    model.forward(state, 0, 0);  // warm-up, as the reference (src/main.cpp:72)

    std::vector<int> encoding = tokenizer.encode(prompt, true);
    const size_t n_prompt = encoding.size();
    const auto t0 = clk::now();
    size_t read_bytes = 0;
    // the hydrate loop (src/main.cpp:94-100) as one xh_prefill call
    model.prefill(state, encoding, 0);
    for (size_t pos = 0; pos < encoding.size(); pos++) read_bytes += model.active_bytes(pos);
    const auto t1 = clk::now();
    if (device_loop && num_steps > 0) {
        const std::vector<int> gen = model.decode_greedy((int)encoding.size(), num_steps, tokenizer.eos_id,
                                                         tokenizer.eot_id);
        for (int t : gen) {
            std::cout << tokenizer.decode_one(encoding.back(), t) << std::flush;
            encoding.push_back(t);
            read_bytes += model.active_bytes(encoding.size() - 1);
        }
    } else {
        for (int i = 0; i < num_steps || num_steps == -1; i++) {
            const int token_id = sampler.sample_argmax(state);
            std::cout << tokenizer.decode_one(encoding.back(), token_id) << std::flush;
            encoding.push_back(token_id);
            if (token_id == tokenizer.eos_id || token_id == tokenizer.eot_id) break;
            model.forward(state, token_id, (int)encoding.size() - 1);
            read_bytes += model.active_bytes(encoding.size() - 1);
        }
    }
    const auto t2 = clk::now();
    std::cout << "\n" << std::endl;
    const double elapsed = secs(t0, t2), decode = secs(t1, t2);
    const size_t gen = encoding.size() - n_prompt;
    printf("Generation stats (wall clock):\n  %zu tokens (%zu prompt + %zu generated)\n  throughput: %.5g tok/s\n"
           "  decode: %.5g tok/s\n  hydrate: %.5gs\n  bandwidth: %.5g GB/s\n  total: %.5gs\n",
           encoding.size(), n_prompt, gen, encoding.size() / elapsed, gen ? gen / decode : 0.0, secs(t0, t1),
           (double)read_bytes / 1e9 / elapsed, elapsed);
    print_ids(encoding);
}

// run_perplexity, src/main.cpp:198-268
static void run_perplexity(const std::string& path, Device dev, const std::string& prompt, int context) {
    const XalmFile file = XalmFile::load(path);
    const Model model = Model::from_xalm(file, context, dev);
    InferenceState state(model.config);
    const Tokenizer tokenizer(file);
    model.forward(state, 0, 0);
    const std::vector<int> encoding = tokenizer.encode(prompt, true);
    double sum_logprob = 0.0, ss_logprob = 0.0;
    const size_t N = encoding.size() - 1;
    const auto t0 = clk::now();
    // the forward + sample_prob loop runs on the device (logits never cross to the host); the
    // log and the double sums stay here, as in the reference
    const std::vector<float> probs = model.token_probs(encoding, 0);
    for (size_t pos = 0; pos < N; pos++) {
        const double logprob = std::log(probs[pos]);
        sum_logprob += logprob;
        ss_logprob += logprob * logprob;
    }
    const double elapsed = secs(t0, clk::now());
    const double ppl = std::exp(-sum_logprob / N);
    const double err = ppl * std::sqrt((ss_logprob - sum_logprob * sum_logprob / N) / N / N);
    printf("Stats:\n  %zu tokens\n  perplexity: %.5g +- %.5g\n  throughput: %.5g tok/s\n  total: %.5gs\n", N, ppl, err,
           N / elapsed, elapsed);
    printf("perplexity: %.9g\n", ppl);
}

int main(int argc, char** argv) {
    std::string path, mode = "completion", prompt = "Q: What is the meaning of life? A:", prompt_path;
    std::string device = "hip";
    int context = 0, num_steps = 128, device_loop = 0;
    if (argc >= 2) path = argv[1];
    else error_usage();
    for (int i = 2; i < argc;) {
        if (i + 1 >= argc || argv[i][0] != '-' || strlen(argv[i]) != 2) error_usage();
        const char f = argv[i][1];
        const std::string v = argv[i + 1];
        if (f == 'm') {
            if (std::string("completion").rfind(v, 0) == 0) mode = "completion";
            else if (std::string("perplexity").rfind(v, 0) == 0) mode = "perplexity";
            else error_usage();
        } else if (f == 'd') {
            if (std::string("hip").rfind(v, 0) == 0 || std::string("cuda").rfind(v, 0) == 0) device = "hip";
            else if (std::string("cpu").rfind(v, 0) == 0) device = "cpu";
            else error_usage();
        } else if (f == 'i') prompt = v;
        else if (f == 'f') prompt_path = v;
        else if (f == 'T') context = std::stoi(v);
        else if (f == 'n') num_steps = std::stoi(v);
        else if (f == 'g') device_loop = std::stoi(v);
        else error_usage();
        i += 2;
    }
    if (!prompt_path.empty()) {
        std::ifstream file(prompt_path);
        if (!file.is_open()) {
            std::cerr << "Error: could not open file " << prompt_path << std::endl;
            return 1;
        }
        std::stringstream buffer;
        buffer << file.rdbuf();
        prompt = buffer.str();
    }
    const Device dev = device == "cpu" ? Device::CPU : Device::HIP;
    try {
        if (mode == "completion") run_completion(path, dev, prompt, context, num_steps, device_loop != 0);
        else run_perplexity(path, dev, prompt, context);
    } catch (const std::exception& e) {
        fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
