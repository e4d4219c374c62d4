// skq — the reference's command line (src/main.cpp:24-276) on the MI355X path:
//   skq [-h] [-k K1,K2,...] [-o index|quant] <args>
//   -o index <reference.fasta> <index_output>
//   -o quant <index_file> <reads.fastq> <output.csv>     (the default mode)
// index: FASTA -> per-transcript FracMinHash sketches -> inverted index -> the legacy file, plus
//        its compact CSR sidecar <index>.skq (loaded by quant when its stamp matches).
// quant: legacy file -> device index; FASTQ streamed to the GPU, parsed there and mapped in
//        batches (skq_ingest: sketch + sparse chain); the last valid record of every read id
//        kept; EM (20 rounds, 0.01) and assignment on the GPU -> CSV. As in the reference, quant uses the index's k list.
#include <getopt.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>
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
              << "Environment: SKQ_DEVICE (GPU ordinal, default 0), SKQ_BATCH (reads per batch),\n"
              << "             SKQ_CHUNK_MB (FASTQ MiB per device chunk, default 64).\n";
}

const float kSketchSize = 0.05f;  // src/main.cpp:43

int device() {
    const char* e = std::getenv("SKQ_DEVICE");
    return e ? std::atoi(e) : 0;
}

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
    skq_index* ix = nullptr;
    check(skq_index_from_tables(device(), ntx, nk, ks, tabs, &ix), "device index");

    uint64_t batch = 1u << 21;  // reads per batch (2M and 64-MiB chunks: tools/ingest_bench.py sweep)
    if (const char* e = std::getenv("SKQ_BATCH")) batch = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10));
    skq_session* s = nullptr;
    check(skq_session_create(ix, batch, 256, &s), "session");
    // FASTQ parsed on the GPU: the reader thread streams the file to HBM (skq_ingest)
    skq_ingest* q = nullptr;
    uint64_t chunk = 0;
    if (const char* e = std::getenv("SKQ_CHUNK_MB")) chunk = std::strtoull(e, nullptr, 10) << 20;
    check(skq_ingest_open(s, reads_path.c_str(), chunk, 8, &q), "FASTQ");

    // every record's candidates stay on the device, appended batch by batch to the EM set
    skq_em_set* em = nullptr;
    check(skq_em_create(device(), ntx, &em), "EM");
    const uint32_t thr = skq_threshold((double)kSketchSize);
    for (;;) {
        uint64_t n = 0, first = 0;
        check(skq_ingest_map(q, thr, 0.9, 0, nullptr, &n, &first), "sketch + sparse chain");
        if (n == 0) break;
        check(skq_em_add_session(em, s, nullptr), "EM reads");
    }
    std::vector<uint8_t> kept(skq_ingest_records(q));
    check(skq_ingest_finish(q, kept.data()), "duplicate reads");
    std::cout << "Loading read completed" << std::endl;
    std::cout << "Sparse chaining completed" << std::endl;

    // the reads sparse_chain saw: status OK, and the last such record of their id
    check(skq_em_select(em, kept.data()), "EM reads");
    std::vector<double> pi(ntx), counts(ntx);
    std::vector<uint8_t> assigned(ntx);
    int iters = 0;
    check(skq_em_run(em, 20, 0.01, pi.data(), &iters), "EM");
    std::cout << "EM estimation completed" << std::endl;
    check(skq_em_assign_host(em, nullptr, counts.data(), assigned.data()), "assign");
    std::cout << "Read assignment completed" << std::endl;
    check(skq_csv_write(out_path.c_str(), tx, counts.data(), assigned.data(), pi.data()), "output_to_csv");
    std::cout << "Output written to " << out_path << std::endl;
    skq_em_free(em);
    skq_ingest_close(q);
    skq_session_free(s);
    skq_index_free(ix);
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
