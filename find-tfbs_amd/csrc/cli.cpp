// find-tfbs-amd: the find-tfbs command line (main.rs:163-232) over tfbs_run.
// Long flags are the reference's; the short ones it binds twice (-n, -t,
// main.rs:174/179, 177/181) are accepted in their first meaning only.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/tfbs_amd.h"

static void usage() {
    fprintf(stderr,
            "find-tfbs-amd 1.0.1 (MI355X)\nFind patterns in a VCF file\n\n"
            "USAGE: find-tfbs-amd --chromosome CHROM --input IN --output OUT --reference REF --bed BED[,BED..]\n"
            "       --pwm_names N1[,N2..] --pwm_file PWM --pwm_threshold_directory DIR --pwm_threshold T\n"
            "       [--forward_only] [--threads N] [--min_maf N] [--after_position P] [--samples FILE]\n"
            "       [--tabix] [--verbose] [--device D | --devices D1,D2,.. | --gpus N] [--regions_per_batch N]\n"
            "  --devices: one contiguous block of merged regions per listed HIP device (a device may repeat);\n"
            "  --gpus N: devices 0..N-1.  The output is the same for any device list.\n");
}

int main(int argc, char **argv) {
    tfbs_run_args a;
    memset(&a, 0, sizeof a);
    a.threads = 1;
    bool have_thr = false;
    std::string gpus;
    for (int i = 1; i < argc; i++) {
        std::string k = argv[i];
        auto val = [&](const char *name) -> const char * {
            if (i + 1 >= argc) {
                fprintf(stderr, "error: %s needs a value\n", name);
                exit(2);
            }
            return argv[++i];
        };
        if (k == "--chromosome" || k == "-c") a.chromosome = val("--chromosome");
        else if (k == "--input" || k == "-i") a.bcf = val("--input");
        else if (k == "--output" || k == "-o") a.output = val("--output");
        else if (k == "--reference" || k == "-r") a.reference = val("--reference");
        else if (k == "--bed" || k == "-b") a.bed_files = val("--bed");
        else if (k == "--pwm_names" || k == "-n") a.pwm_names = val("--pwm_names");
        else if (k == "--pwm_file" || k == "-p") a.pwm_file = val("--pwm_file");
        else if (k == "--pwm_threshold_directory") a.pwm_threshold_dir = val(k.c_str());
        else if (k == "--pwm_threshold" || k == "-t") {
            a.pwm_threshold = strtof(val(k.c_str()), nullptr);
            have_thr = true;
        } else if (k == "--forward_only" || k == "-f") a.forward_only = 1;
        else if (k == "--threads") {
            long n = strtol(val(k.c_str()), nullptr, 10);
            if (n < 1) {
                fprintf(stderr, "Wrong number of threads\n");
                return 2;
            }
            a.threads = (uint32_t)n;
        } else if (k == "--min_maf" || k == "-m") a.min_maf = (uint32_t)strtoul(val(k.c_str()), nullptr, 10);
        else if (k == "--after_position") a.after_position = strtoull(val(k.c_str()), nullptr, 10);
        else if (k == "--samples" || k == "-s") a.samples_file = val(k.c_str());
        else if (k == "--tabix" || k == "-z") a.tabix = 1;
        else if (k == "--verbose" || k == "-v") a.verbose = 1;
        else if (k == "--device") a.device = atoi(val(k.c_str()));
        else if (k == "--devices") a.devices = val(k.c_str());
        else if (k == "--gpus") {
            long n = strtol(val(k.c_str()), nullptr, 10);
            if (n < 1) {
                fprintf(stderr, "Wrong number of GPUs\n");
                return 2;
            }
            gpus.clear();
            for (long d = 0; d < n; d++) gpus += (d ? "," : "") + std::to_string(d);
            a.devices = gpus.c_str();
        }
        else if (k == "--regions_per_batch") a.regions_per_batch = (uint32_t)strtoul(val(k.c_str()), nullptr, 10);
        else if (k == "--help" || k == "-h") {
            usage();
            return 0;
        } else {
            fprintf(stderr, "error: unexpected argument '%s'\n", k.c_str());
            usage();
            return 2;
        }
    }
    if (!a.chromosome || !a.bcf || !a.output || !a.reference || !a.bed_files || !a.pwm_names || !a.pwm_file ||
        !a.pwm_threshold_dir || !have_thr) {
        usage();
        return 2;
    }
    int rc = tfbs_run(&a);
    if (rc) {
        fprintf(stderr, "find-tfbs-amd: %s (%s)\n", tfbs_last_error(), tfbs_strerror(rc));
        return 101;  // a Rust panic's exit status
    }
    printf("End of program.\n");
    return 0;
}
