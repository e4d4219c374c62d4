// skq — the reference's command line (src/main.cpp:24-276) on the MI355X path:
//   skq [-h] [-k K1,K2,...] [-o index|quant] <args>
//   -o index <reference.fasta> <index_output>
//   -o quant <index_file> <reads.fastq> <output.csv>     (the default mode)
// index: FASTA -> per-transcript FracMinHash sketches -> inverted index -> the legacy file, plus
//        its compact CSR sidecar <index>.skq (loaded by quant when its stamp matches).
// quant: legacy file -> device index; FASTQ streamed to the GPU, parsed there and mapped in
//        batches (skq_ingest: sketch + sparse chain); the last valid record of every read id
//        kept; EM (20 rounds, 0.01) and assignment on the GPU -> CSV. As in the reference, quant uses the index's k list.
//        Several GPUs (SKQ_DEVICES=0,1,...): the file is split into one part per device at line
//        starts (skq_fastq_split), each device holds the index and maps its part on a host thread
//        of its own, duplicate ids are settled across the parts (skq_ingest_supersede), and every
//        EM round is the devices' E-steps, one RCCL all-reduce of the posterior sums over xGMI,
//        and the same M-step on every device (src/main.cpp:165-197, src/isoform_assignment.cpp).
#include <getopt.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "skq.h"
#include "skq_host.h"

namespace {

void check(int rc, const char* what) {
    if (rc != 0) throw std::runtime_error(std::string(what) + ": " + skq_last_error());
}

void print_help(const std::string& prog) {
    std::cout << "Usage: " << prog << " [OPTIONS] <mode> [arguments]\n"
              << "Modes:\n"
              << "  index   Build index from reference genome\n"
              << "  quant   Quantify using pre-built index and reads\n\n"
              << "Options:\n"
              << "  -h, --help              Show this help message and exit\n"
              << "  -k, --kmer-length SIZE  Comma separated list of k-mer lengths (default: 31)\n"
              << "  -o, --mode MODE         Mode: index or quant (default: quant)\n\n"
              << "Index mode usage:\n"
              << "  " << prog << " -o index <reference_genome.fasta> <index_output>\n\n"
              << "Quant mode usage:\n"
              << "  " << prog << " -o quant <index_file> <reads.fastq> <output>\n\n"
              << "Environment: SKQ_DEVICE (GPU ordinal, default 0), SKQ_DEVICES (GPU list for quant,\n"
              << "             e.g. 0,1,2,3 or all), SKQ_BATCH (reads per batch), SKQ_CHUNK_MB (FASTQ MiB\n"
              << "             per device chunk, default 64), SKQ_REDUCE (rccl | host: how the EM sums\n"
              << "             reduce over devices; rccl on one device runs the sharded EM over a\n"
              << "             one-rank RCCL communicator).\n";
}

const float kSketchSize = 0.05f;  // src/main.cpp:43

int device() {
    const char* e = std::getenv("SKQ_DEVICE");
    return e ? std::atoi(e) : 0;
}

// quant's devices: SKQ_DEVICES (a list, or "all"), else SKQ_DEVICE
std::vector<int> devices() {
    const char* e = std::getenv("SKQ_DEVICES");
    if (!e || !*e) return {device()};
    std::vector<int> d;
    if (std::string(e) == "all") {
        for (int i = 0; i < skq_device_count(); ++i) d.push_back(i);
    } else {
        std::istringstream iss(e);
        std::string tok;
        while (std::getline(iss, tok, ','))
            if (!tok.empty()) d.push_back(std::stoi(tok));
    }
    if (d.empty()) throw std::runtime_error("SKQ_DEVICES names no device");
    return d;
}

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// One device's share of quant: its copy of the index, a session, the GPU ingest of its part of
// the FASTQ file, and the candidate lists kept on the device for the EM.
struct Part {
    int dev = 0;
    uint64_t lo = 0, hi = 0;
    uint32_t state = 0;
    skq_index* ix = nullptr;
    skq_session* s = nullptr;
    skq_ingest* q = nullptr;
    skq_em_set* em = nullptr;
    std::vector<uint8_t> kept;
    hipStream_t st = nullptr;
    double *d_pi = nullptr, *d_post = nullptr;
    uint8_t* d_assigned = nullptr;
    std::string err;

    void map(const std::string& reads_path, uint32_t ntx, uint32_t nk, const uint32_t* ks, const skq_tables* tabs,
             const skq_seqs* tx) {
        // (one k: the chained tables from the index's transcripts)
        check(skq_index_from_tables_chained(dev, ntx, nk, ks, tabs, tx, skq_threshold((double)kSketchSize), &ix),
              "device index");
        uint64_t batch = 1u << 21;  // reads per batch (2M and 64-MiB chunks: tools/ingest_bench.py sweep)
        if (const char* e = std::getenv("SKQ_BATCH")) batch = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10));
        check(skq_session_create(ix, batch, 256, &s), "session");
        uint64_t chunk = 0;
        if (const char* e = std::getenv("SKQ_CHUNK_MB")) chunk = std::strtoull(e, nullptr, 10) << 20;
        check(skq_ingest_open_range(s, reads_path.c_str(), lo, hi, state, chunk, 0, &q), "FASTQ");
        // every record's candidates stay on the device, appended batch by batch to the EM set
        check(skq_em_create(dev, ntx, &em), "EM");
        const uint32_t thr = skq_threshold((double)kSketchSize);
        for (;;) {
            uint64_t n = 0, first = 0;
            check(skq_ingest_map(q, thr, 0.9, 0, nullptr, &n, &first), "sketch + sparse chain");
            if (n == 0) break;
            check(skq_em_add_session(em, s, nullptr), "EM reads");
        }
        kept.resize(skq_ingest_records(q));
        check(skq_ingest_finish(q, kept.data()), "duplicate reads");
    }

    ~Part() {
        if (d_pi) skq_free(d_pi);
        if (d_post) skq_free(d_post);
        if (d_assigned) skq_free(d_assigned);
        if (st) (void)hipStreamDestroy(st);
        skq_em_free(em);
        skq_ingest_close(q);
        skq_session_free(s);
        skq_index_free(ix);
    }
};

// SKQ_REDUCE: "rccl" forces the sharded EM and RCCL even on one device (a one-rank communicator:
// the library path the multi-GPU run takes, testable on a one-GPU box); "host" forces the
// host-staged sums; unset: RCCL when the devices are distinct, the host when one repeats
std::string reduce_mode() {
    const char* e = std::getenv("SKQ_REDUCE");
    return e ? std::string(e) : std::string();
}

// Sum (or max) of one device array over the parts, left in every part's copy: RCCL over xGMI
// when the devices are distinct; a host-staged sum in part order when a device repeats (several
// parts sharing one GPU, as the tests run them).
struct Reducer {
    std::vector<Part*> parts;
    std::vector<ncclComm_t> comms;
    bool host = false;

    explicit Reducer(std::vector<Part*> ps) : parts(std::move(ps)) {
        std::vector<int> devs;
        for (Part* p : parts) devs.push_back(p->dev);
        std::vector<int> u = devs;
        std::sort(u.begin(), u.end());
        host = std::unique(u.begin(), u.end()) != u.end();
        const std::string mode = reduce_mode();
        if (mode == "rccl" && host) throw std::runtime_error("SKQ_REDUCE=rccl needs distinct devices");
        if (mode == "host") host = true;
        if (!host) {
            comms.resize(parts.size());
            if (ncclCommInitAll(comms.data(), (int)devs.size(), devs.data()) != ncclSuccess)
                throw std::runtime_error("RCCL communicator setup failed");
        }
    }
    ~Reducer() {
        for (ncclComm_t c : comms) (void)ncclCommDestroy(c);
    }
    template <typename T>
    void all(T* (Part::*field), size_t count, ncclDataType_t type, ncclRedOp_t op) {
        if (!host) {
            if (ncclGroupStart() != ncclSuccess) throw std::runtime_error("RCCL group");
            for (size_t d = 0; d < parts.size(); ++d) {
                T* p = parts[d]->*field;
                if (ncclAllReduce(p, p, count, type, op, comms[d], parts[d]->st) != ncclSuccess)
                    throw std::runtime_error("RCCL all-reduce failed");
            }
            if (ncclGroupEnd() != ncclSuccess) throw std::runtime_error("RCCL group");
            return;
        }
        std::vector<T> acc(count), h(count);
        for (size_t d = 0; d < parts.size(); ++d) {
            hip_check(hipSetDevice(parts[d]->dev), "device");
            hip_check(hipMemcpyAsync(h.data(), parts[d]->*field, count * sizeof(T), hipMemcpyDeviceToHost, parts[d]->st),
                      "reduce copy");
            hip_check(hipStreamSynchronize(parts[d]->st), "reduce copy");
            for (size_t i = 0; i < count; ++i) acc[i] = d == 0 ? h[i] : (op == ncclSum ? acc[i] + h[i] : std::max(acc[i], h[i]));
        }
        for (Part* p : parts) {
            hip_check(hipSetDevice(p->dev), "device");
            hip_check(hipMemcpyAsync(p->*field, acc.data(), count * sizeof(T), hipMemcpyHostToDevice, p->st), "reduce copy");
            hip_check(hipStreamSynchronize(p->st), "reduce copy");
        }
    }
};

void build_and_save_index(const std::string& fasta, const std::string& out, const std::vector<uint32_t>& ks) {
    const auto t0 = std::chrono::steady_clock::now();
    skq_seqs* tx = nullptr;
    check(skq_fasta_load(fasta.c_str(), &tx), "load_fasta");
    const uint8_t* bytes = nullptr;
    const uint64_t* offs = nullptr;
    check(skq_seqs_view(tx, &bytes, &offs, nullptr, nullptr), "sequences");
    skq_tables* tabs = nullptr;
    // on the GPU when there is one (skq_tables_build_gpu), else on host threads: the same tables
    if (skq_device_count() > device())
        check(skq_tables_build_gpu(device(), (uint32_t)skq_seqs_count(tx), bytes, offs, (uint32_t)ks.size(), ks.data(),
                                   skq_threshold((double)kSketchSize), &tabs),
              "index build");
    else
        check(skq_tables_build((uint32_t)skq_seqs_count(tx), bytes, offs, (uint32_t)ks.size(), ks.data(),
                               skq_threshold((double)kSketchSize), 0, &tabs),
              "index build");
    const std::chrono::duration<double> dt = std::chrono::steady_clock::now() - t0;
    std::cout << "Index built in " << dt.count() << " seconds." << std::endl;
    check(skq_legacy_index_write(out.c_str(), (uint32_t)ks.size(), ks.data(), tx, tabs), "save_index");
    // the compact CSR copy quant loads instead of parsing the legacy file (skq_index_open)
    check(skq_sidecar_write(out.c_str(), (uint32_t)ks.size(), ks.data(), tx, tabs), "index sidecar");
    std::cout << "Index saved to " << out << std::endl;
    skq_tables_free(tabs);
    skq_seqs_free(tx);
}

void quantification(const std::string& index_path, const std::string& reads_path, const std::string& out_path) {
    skq_legacy_index* lx = nullptr;
    check(skq_index_open(index_path.c_str(), &lx, nullptr), "load_index");
    std::cout << "Index loaded from " << index_path << std::endl;
    std::cout << "Loading index completed" << std::endl;
    uint32_t nk = 0;
    const uint32_t* ks = nullptr;
    const skq_seqs* tx = nullptr;
    const skq_tables* tabs = nullptr;
    check(skq_legacy_index_view(lx, &nk, &ks, &tx, &tabs), "index view");
    if (nk == 0) throw std::runtime_error("the index holds no k-mer lengths");
    const uint32_t ntx = (uint32_t)skq_seqs_count(tx);

    // one part of the file per device, mapped on a host thread each
    const std::vector<int> devs = devices();
    const uint32_t D = (uint32_t)devs.size();
    std::vector<uint64_t> offs(D + 1);
    std::vector<uint32_t> states(D);
    check(skq_fastq_split(reads_path.c_str(), D, offs.data(), states.data()), "FASTQ split");
    std::vector<Part> parts(D);
    for (uint32_t d = 0; d < D; ++d) {
        parts[d].dev = devs[d];
        parts[d].lo = offs[d];
        parts[d].hi = offs[d + 1];
        parts[d].state = states[d];
    }
    {
        std::vector<std::thread> ts;
        for (Part& p : parts)
            ts.emplace_back([&p, &reads_path, ntx, nk, ks, tabs, tx] {
                try {
                    hip_check(hipSetDevice(p.dev), "device");
                    p.map(reads_path, ntx, nk, ks, tabs, tx);
                } catch (const std::exception& e) {
                    p.err = e.what();
                }
            });
        for (auto& t : ts) t.join();
    }
    for (Part& p : parts)
        if (!p.err.empty()) throw std::runtime_error(p.err);
    std::vector<skq_ingest*> qs;
    std::vector<uint8_t*> kp;
    for (Part& p : parts) {
        qs.push_back(p.q);
        kp.push_back(p.kept.data());
    }
    check(skq_ingest_supersede(qs.data(), D, kp.data()), "duplicate reads");  // (one part: no-op)
    std::cout << "Loading read completed" << std::endl;
    std::cout << "Sparse chaining completed" << std::endl;

    // the reads sparse_chain saw: status OK, and the last such record of their id
    uint64_t R = 0;
    for (Part& p : parts) {
        check(skq_em_select(p.em, p.kept.data()), "EM reads");
        R += skq_em_reads(p.em);
    }
    std::vector<double> pi(ntx), counts(ntx);
    std::vector<uint8_t> assigned(ntx);
    if (D == 1 && reduce_mode() != "rccl") {
        Part& p = parts[0];
        int iters = 0;
        check(skq_em_run(p.em, 20, 0.01, pi.data(), &iters), "EM");
        std::cout << "EM estimation completed" << std::endl;
        check(skq_em_assign_host(p.em, nullptr, counts.data(), assigned.data()), "assign");
    } else {
        // sharded rounds (src/isoform_assignment.cpp:9-70): every device's E-step over its reads,
        // the posterior sums all-reduced, the same M-step (and convergence test) on every device
        std::vector<Part*> pp;
        for (Part& p : parts) {
            hip_check(hipSetDevice(p.dev), "device");
            hip_check(hipStreamCreateWithFlags(&p.st, hipStreamNonBlocking), "stream");
            check(skq_malloc(p.dev, ntx * 8ull, reinterpret_cast<void**>(&p.d_pi)), "EM buffers");
            check(skq_malloc(p.dev, ntx * 8ull, reinterpret_cast<void**>(&p.d_post)), "EM buffers");
            check(skq_malloc(p.dev, ntx, reinterpret_cast<void**>(&p.d_assigned)), "EM buffers");
            check(skq_em_init(p.em, p.d_pi, p.st), "EM");
            pp.push_back(&p);
        }
        Reducer red(pp);
        int it = 0;
        for (; it < 20; ++it) {
            for (Part& p : parts) check(skq_em_estep(p.em, p.d_pi, p.d_post, p.st), "EM");
            red.all(&Part::d_post, ntx, ncclDouble, ncclSum);
            double change = 0.0;
            for (Part& p : parts) check(skq_em_mstep(p.em, p.d_pi, p.d_post, R, &change, p.st), "EM");
            if (change < 0.01) {  // (:62-64; the same value on every device)
                ++it;
                break;
            }
        }
        std::cout << "EM estimation completed" << std::endl;
        // assignment: counts summed over the devices, assigned flags or-ed (max)
        for (Part& p : parts) check(skq_em_assign(p.em, p.d_pi, p.d_post, p.d_assigned, p.st), "assign");
        red.all(&Part::d_post, ntx, ncclDouble, ncclSum);
        red.all(&Part::d_assigned, ntx, ncclUint8, ncclMax);
        for (Part& p : parts) check(skq_stream_sync(p.st), "assign");
        hip_check(hipSetDevice(parts[0].dev), "device");
        check(skq_memcpy_d2h(pi.data(), parts[0].d_pi, ntx * 8ull, parts[0].st), "assign");
        check(skq_memcpy_d2h(counts.data(), parts[0].d_post, ntx * 8ull, parts[0].st), "assign");
        check(skq_memcpy_d2h(assigned.data(), parts[0].d_assigned, ntx, parts[0].st), "assign");
    }
    std::cout << "Read assignment completed" << std::endl;
    check(skq_csv_write(out_path.c_str(), tx, counts.data(), assigned.data(), pi.data()), "output_to_csv");
    std::cout << "Output written to " << out_path << std::endl;
    parts.clear();
    skq_legacy_index_free(lx);
}

}  // namespace

int main(int argc, char* argv[]) {
    std::string mode = "quant";
    std::vector<uint32_t> ks = {31};
    static struct option long_options[] = {{"help", no_argument, 0, 'h'},
                                           {"kmer-length", required_argument, 0, 'k'},
                                           {"mode", required_argument, 0, 'o'},
                                           {0, 0, 0, 0}};
    int opt, option_index = 0;
    while ((opt = getopt_long(argc, argv, "hk:o:", long_options, &option_index)) != -1) {
        switch (opt) {
        case 'h':
            print_help(argv[0]);
            return 0;
        case 'k': {
            ks.clear();
            std::istringstream iss(optarg);
            std::string tok;
            while (std::getline(iss, tok, ','))
                if (!tok.empty()) ks.push_back((uint32_t)std::stoul(tok));
            break;
        }
        case 'o':
            mode = optarg;
            break;
        default:
            print_help(argv[0]);
            return 1;
        }
    }
    try {
        if (mode == "index") {
            if (optind + 2 > argc) {
                std::cerr << "Usage: " << argv[0] << " index <reference_genome.fasta> <index_output>" << std::endl;
                return 1;
            }
            build_and_save_index(argv[optind], argv[optind + 1], ks);
        } else if (mode == "quant") {
            if (optind + 3 > argc) {
                std::cerr << "Usage: " << argv[0] << " quant <index_file> <reads.fastq> <output>" << std::endl;
                return 1;
            }
            quantification(argv[optind], argv[optind + 1], argv[optind + 2]);
        } else {
            std::cerr << "Invalid mode. Please choose 'index' or 'quant'." << std::endl;
            return 1;
        }
    } catch (const std::exception& e) {
        std::cerr << "skq: " << e.what() << std::endl;
        return 1;
    }
    return 0;
}
