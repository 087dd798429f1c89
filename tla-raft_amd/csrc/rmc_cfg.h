// rmc_cfg.h -- TLC model-config parsing for Raft.cfg (host only).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "rmc.h"

namespace rmc {

struct ParsedModel {
    rmc_config cfg{};
    std::vector<std::string> servers, vals;   // model-value names in TLC order
    std::vector<std::string> invariant_names; // as written in the cfg
    std::vector<std::string> ignored_constants;
    std::string module = "Raft";
    bool symmetry = false, view = false;
    int check_deadlock_cfg = -1;              // CHECK_DEADLOCK in the cfg (-1 = absent)
};

uint64_t fnv1a_spec(const std::string &text);
bool parse_model(const std::string &cfg_text, const char *tla_text, ParsedModel *pm, std::string &err);

}  // namespace rmc
