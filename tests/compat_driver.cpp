// compat_driver.cpp -- test driver for libturbo_logmap_compat.so.  Plays ITTC/main.cpp's part:
// defines the main.h globals and calls the reference's C++ entry points in main.cpp's order.
//   compat_driver encode K f1 f2 src.bin coded.bin          TurboEnCoding (host only)
//   compat_driver awgn   n sigma seed send.bin r.bin          srand(seed); AWGN (host only)
//   compat_driver decode K f1 f2 nframes flow.bin out.bin     TurboCodingInit; per frame
//        TurboDecoding (flow scaled x0.5 in place, written back after out); TurboCodingRelease
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

int source_length, MODULATION, length_after_code, f1, f2, SYMBOL_NUM;   // ITTC/main.h:6-11
extern int M_num_reg;

void TurboCodingInit();
void TurboEnCoding(int* source, int* coded_source, int source_length);
void AWGN(double* send, double* r, double sigma, int totallength);
void TurboDecoding(double* flow_for_decode, int* flow_decoded, int flow_length);
void TurboCodingRelease();

template <typename T>
static std::vector<T> slurp(const char* path, size_t n)
{
    std::vector<T> v(n);
    FILE* f = std::fopen(path, "rb");
    if (!f || std::fread(v.data(), sizeof(T), n, f) != n) {
        std::fprintf(stderr, "read %s failed\n", path);
        std::exit(2);
    }
    std::fclose(f);
    return v;
}

template <typename T>
static void spill(const char* path, const T* p, size_t n, const char* mode = "wb")
{
    FILE* f = std::fopen(path, mode);
    if (!f || std::fwrite(p, sizeof(T), n, f) != n) {
        std::fprintf(stderr, "write %s failed\n", path);
        std::exit(2);
    }
    std::fclose(f);
}

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    if (!std::strcmp(argv[1], "encode") && argc == 7) {
        source_length = std::atoi(argv[2]);
        f1 = std::atoi(argv[3]);
        f2 = std::atoi(argv[4]);
        std::vector<int> src = slurp<int>(argv[5], source_length);
        std::vector<int> coded(3 * source_length + 4 * M_num_reg);
        TurboEnCoding(src.data(), coded.data(), source_length);
        spill(argv[6], coded.data(), coded.size());
        return 0;
    }
    if (!std::strcmp(argv[1], "awgn") && argc == 7) {
        const int n = std::atoi(argv[2]);
        const double sigma = std::atof(argv[3]);
        std::srand((unsigned)std::atoi(argv[4]));
        std::vector<double> send = slurp<double>(argv[5], n), r(n);
        AWGN(send.data(), r.data(), sigma, n);
        spill(argv[6], r.data(), r.size());
        return 0;
    }
    if (!std::strcmp(argv[1], "decode") && argc == 8) {
        source_length = std::atoi(argv[2]);
        f1 = std::atoi(argv[3]);
        f2 = std::atoi(argv[4]);
        const int nf = std::atoi(argv[5]);
        const int n = 3 * source_length + 4 * M_num_reg;
        std::vector<double> flow = slurp<double>(argv[6], (size_t)nf * n);
        std::vector<int> out(15 * (size_t)source_length);
        TurboCodingInit();
        std::remove(argv[7]);
        for (int fr = 0; fr < nf; ++fr) {
            TurboDecoding(flow.data() + (size_t)fr * n, out.data(), n);
            spill(argv[7], out.data(), out.size(), "ab");
        }
        TurboCodingRelease();
        std::string p = std::string(argv[7]) + ".flow";
        spill(p.c_str(), flow.data(), flow.size());
        return 0;
    }
    std::fprintf(stderr, "bad arguments\n");
    return 2;
}
