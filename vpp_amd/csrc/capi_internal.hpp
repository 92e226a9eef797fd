// Handle types behind the C ABI (include/policygpu.h), shared by capi.cpp and capi_cfg.cpp.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "../../include/policygpu.h"
#include "configurator.hpp"
#include "engine.hpp"

struct pg_ctx {
    pg::Engine eng;
};
struct pg_renderer {
    pg_ctx* ctx;
    std::unique_ptr<pg::Renderer> r;
};
struct pg_txn {
    pg_ctx* ctx;
    std::unique_ptr<pg::RendererTxn> t;
};
struct pg_mock_renderer {
    pg::MockRenderer r;
};
struct pg_configurator {
    pg::PolicyConfigurator c;
    std::vector<std::unique_ptr<pg::CfgRenderer>> adapters;  // GPU renderers seen as configurator sinks
    std::string last_error;
};
struct pg_cfg_txn {
    pg_configurator* c;
    std::unique_ptr<pg::PolicyConfiguratorTxn> t;
};

namespace pg {
// pg_ipnet <-> net.IPNet (IPv4: 4-byte address and mask, as net.ParseCIDR returns them)
IPNet to_ipnet(const pg_ipnet& n);
pg_ipnet to_pg_ipnet(const IPNet& n);
}  // namespace pg
