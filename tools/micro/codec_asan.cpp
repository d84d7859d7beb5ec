// Host sanitizer harness for the watch-event codec (kwok_amd/csrc/codec.cpp): decodes a file of
// length-prefixed documents (tools/codec_asan.sh writes golden + mutated ones) with 4 threads.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kwok_engine.h"
int main(int argc, char** argv) {
    FILE* f = fopen(argc > 1 ? argv[1] : "/tmp/asan/docs.bin", "rb");
    if (!f) return 3;
    std::vector<char> all; std::vector<uint64_t> off; std::vector<uint32_t> len;
    uint32_t n;
    while (fread(&n, 4, 1, f) == 1) { off.push_back(all.size()); len.push_back(n); size_t s = all.size(); all.resize(s + n); if (fread(all.data() + s, 1, n, f) != n) return 4; }
    kwok_codec_config cfg{1, "", "", "fake=custom,a in (b,c)", "!x"};
    kwok_codec* c; if (kwok_codec_create(&cfg, &c)) return 2;
    std::vector<kwok_pod_doc> out(off.size()); std::vector<int32_t> st(off.size());
    int bad = kwok_decode_pods(c, all.data(), all.size(), off.data(), len.data(), off.size(), 4, out.data(), st.data());
    std::vector<kwok_node_event> ne(off.size());
    int bad2 = kwok_decode_nodes(c, all.data(), all.size(), off.data(), len.data(), off.size(), 4, ne.data(), st.data());
    printf("docs %zu rejected pods %d nodes %d\n", off.size(), bad, bad2);
    kwok_codec_destroy(c);
    return 0;
}
