// whisper_tokenize: the initial prompt the reference builds from the custom
// vocabulary and the previous chunk's text (src-tauri/src/whisper.rs:97-109) is tokenised by
// whisper.cpp's own tokenizer [ext `tokenize`]: a GPT-2 style regex pre-split followed by greedy
// longest-prefix matching against the model file's vocabulary (no BPE merges). Host-side: the
// prompt is at most a few hundred bytes per call.
//
// Attribution: the pre-split regex and the longest-prefix loop follow whisper.cpp's `tokenize()`
// (https://github.com/ggerganov/whisper.cpp, MIT License, Copyright (c) 2023-2024 The ggml
// authors); bit-exact prompt token ids require the same std::regex semantics.
#include <regex>

#include "engine.h"

namespace wm {

std::vector<int> tokenize(const Vocab& vocab, const std::string& text) {
    static const std::regex re(
        R"('s|'t|'re|'ve|'m|'ll|'d| ?[[:alpha:]]+| ?[[:digit:]]+| ?[^\s[:alpha:][:digit:]]+|\s+(?!\S)|\s+)");
    std::vector<std::string> words;
    std::string str = text;
    std::smatch m;
    while (std::regex_search(str, m, re)) {
        for (auto x : m) words.push_back(x);
        str = m.suffix();
    }
    std::vector<int> tokens;
    for (const auto& word : words) {
        if (word.empty()) continue;
        int i = 0;
        const int n = (int)word.size();
        while (i < n) {
            int j = n;
            bool found = false;
            while (j > i) {
                auto it = vocab.token_to_id.find(word.substr(i, j - i));
                if (it != vocab.token_to_id.end()) {
                    tokens.push_back(it->second);
                    i = j;
                    found = true;
                    break;
                }
                --j;
            }
            if (!found) ++i;  // whisper.cpp logs "unknown token" and skips the byte
        }
    }
    return tokens;
}

}  // namespace wm
