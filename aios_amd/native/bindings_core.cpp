// pybind11 module `aios_amd._core`: the native control-plane cores (tools, memory, orchestrator
// stores, planner / LLM-output parsing) for the asyncio gRPC services in aios_amd/services.
// JSON values cross as native Python objects (dict/list/str/int/float/bool/None); tool I/O stays
// JSON text because the wire format (ExecuteResponse.output_json) is bytes.  Blocking calls
// (tool execution, SQLite) release the GIL.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "gateway.h"
#include "json.h"
#include "memory.h"
#include "orchestrator.h"
#include "security.h"
#include "tools.h"
#include "util.h"

namespace py = pybind11;
using namespace aiosn;

namespace {

Json to_json(const py::handle& o) {
  if (o.is_none()) return Json();
  if (py::isinstance<py::bool_>(o)) return Json(o.cast<bool>());
  if (py::isinstance<py::int_>(o)) return Json((int64_t)o.cast<long long>());
  if (py::isinstance<py::float_>(o)) return Json(o.cast<double>());
  if (py::isinstance<py::str>(o)) return Json(o.cast<std::string>());
  if (py::isinstance<py::bytes>(o)) return Json(o.cast<std::string>());
  if (py::isinstance<py::dict>(o)) {
    Json j = Json::object();
    for (auto kv : o.cast<py::dict>()) j.set(py::str(kv.first).cast<std::string>(), to_json(kv.second));
    return j;
  }
  if (py::isinstance<py::list>(o) || py::isinstance<py::tuple>(o)) {
    Json j = Json::array();
    for (auto v : o) j.push(to_json(v));
    return j;
  }
  throw py::type_error("value is not JSON-serialisable");
}

py::object to_py(const Json& j) {
  switch (j.type()) {
    case Json::NUL: return py::none();
    case Json::BOOL: return py::bool_(j.as_bool());
    case Json::NUM: {
      const double n = j.as_num();
      if ((double)j.as_int() == n && std::abs(n) < 9.0e15) {
        // integral flag is private; integral-valued numbers round-trip as int except floats that
        // were produced as doubles and happen to be whole -- callers treat both the same
        return py::int_(j.as_int());
      }
      return py::float_(n);
    }
    case Json::STR: return py::str(j.as_str());
    case Json::ARR: {
      py::list l;
      for (auto& v : j.as_arr()) l.append(to_py(v));
      return l;
    }
    case Json::OBJ: {
      py::dict d;
      for (auto& kv : j.as_obj()) d[py::str(kv.first)] = to_py(kv.second);
      return d;
    }
  }
  return py::none();
}

py::dict tooldef_py(const ToolDef& d) {
  py::dict o;
  o["name"] = d.name;
  o["namespace"] = d.ns;
  o["version"] = d.version;
  o["description"] = d.description;
  o["required_capabilities"] = d.required_caps;
  o["risk_level"] = d.risk_level;
  o["requires_confirmation"] = d.requires_confirmation;
  o["idempotent"] = d.idempotent;
  o["reversible"] = d.reversible;
  o["timeout_ms"] = d.timeout_ms;
  o["rollback_tool"] = d.rollback_tool;
  o["handler_address"] = d.handler_address;
  o["input_schema"] = d.input_schema;
  return o;
}

ToolDef tooldef_from(const py::dict& o) {
  ToolDef d;
  auto s = [&](const char* k, std::string& dst) {
    if (o.contains(k)) dst = py::str(o[k]).cast<std::string>();
  };
  s("name", d.name);
  s("namespace", d.ns);
  s("version", d.version);
  s("description", d.description);
  s("risk_level", d.risk_level);
  s("rollback_tool", d.rollback_tool);
  s("handler_address", d.handler_address);
  s("input_schema", d.input_schema);
  if (o.contains("required_capabilities")) d.required_caps = o["required_capabilities"].cast<std::vector<std::string>>();
  if (o.contains("requires_confirmation")) d.requires_confirmation = o["requires_confirmation"].cast<bool>();
  if (o.contains("idempotent")) d.idempotent = o["idempotent"].cast<bool>();
  if (o.contains("reversible")) d.reversible = o["reversible"].cast<bool>();
  if (o.contains("timeout_ms")) d.timeout_ms = o["timeout_ms"].cast<int>();
  if (d.version.empty()) d.version = "1.0.0";
  return d;
}

}  // namespace

PYBIND11_MODULE(_core, m) {
  m.doc() = "aiOS MI355X control-plane native core";

  // ---------------------------------------------------------------- helpers
  m.def("sha256_hex", [](const std::string& s) { return sha256_hex(s); });
  m.def("uuid4", &uuid4);
  m.def("json_roundtrip", [](const std::string& s, int indent) { return Json::parse(s).dump(indent); },
        py::arg("text"), py::arg("indent") = -1);
  m.def("hashed_embedding", &hashed_embedding, py::arg("text"), py::arg("dim") = 64);
  m.def("cosine", &cosine);
  m.def("keyword_relevance", &keyword_relevance);
  m.def("estimate_tokens", &estimate_tokens);
  m.def("run_cmd",
        [](const std::vector<std::string>& argv, int timeout_ms, const std::string& stdin_data) {
          CmdLimits lim;
          lim.timeout_ms = timeout_ms;
          lim.stdin_data = stdin_data;
          CmdResult r;
          {
            py::gil_scoped_release rel;
            r = run_cmd(argv, lim);
          }
          py::dict o;
          o["exit_code"] = r.exit_code;
          o["stdout"] = py::bytes(r.out);
          o["stderr"] = py::bytes(r.err);
          o["timed_out"] = r.timed_out;
          return o;
        },
        py::arg("argv"), py::arg("timeout_ms") = 30000, py::arg("stdin_data") = "");
  m.def("sandbox_exec",
        [](const std::string& cmd, const std::vector<std::string>& args, const std::string& input, int timeout_ms,
           size_t mem_bytes) {
          SandboxLimits lim;
          lim.timeout_ms = timeout_ms;
          if (mem_bytes) lim.mem_bytes = mem_bytes;
          SandboxResult r;
          {
            py::gil_scoped_release rel;
            r = sandbox_exec(cmd, args, input, lim);
          }
          py::dict o;
          o["success"] = r.success;
          o["output"] = r.output;
          o["error"] = r.error;
          o["exit_code"] = r.exit_code;
          o["duration_ms"] = r.duration_ms;
          return o;
        },
        py::arg("cmd"), py::arg("args"), py::arg("input") = "", py::arg("timeout_ms") = 30000,
        py::arg("mem_bytes") = 0);
  m.def("should_sandbox", &should_sandbox);
  m.def("plugin_validate", [](const std::string& code) { return to_py(plugin_validate(code)); });
  m.def("plugin_wrapper", &plugin_wrapper);

  // ---------------------------------------------------------------- tools
  py::class_<ToolService>(m, "ToolService")
      .def(py::init([](const std::string& data_dir, const std::string& source_dir) {
             ToolPaths p;
             p.data_dir = data_dir;
             p.source_dir = source_dir;
             return new ToolService(p);
           }),
           py::arg("data_dir"), py::arg("source_dir") = "")
      .def("list_tools",
           [](const ToolService& s, const std::string& ns) {
             py::list l;
             for (auto& d : s.list_tools(ns)) l.append(tooldef_py(d));
             return l;
           },
           py::arg("namespace") = "")
      .def("get_tool",
           [](const ToolService& s, const std::string& name) -> py::object {
             ToolDef d;
             if (!s.get_tool(name, d)) return py::none();
             return tooldef_py(d);
           })
      .def("register_tool",
           [](ToolService& s, const py::dict& def) {
             std::string err;
             const bool ok = s.register_tool(tooldef_from(def), err);
             return py::make_tuple(ok, err);
           })
      .def("deregister_tool", &ToolService::deregister_tool)
      .def("execute",
           [](ToolService& s, const std::string& tool, const std::string& agent, const std::string& task,
              const py::bytes& input_json, const std::string& reason) {
             ExecResult r;
             const std::string in = input_json;
             {
               py::gil_scoped_release rel;
               r = s.execute(tool, agent, task, in, reason);
             }
             py::dict o;
             o["success"] = r.success;
             o["output_json"] = py::bytes(r.output_json);
             o["error"] = r.error;
             o["execution_id"] = r.execution_id;
             o["backup_id"] = r.backup_id;
             o["duration_ms"] = r.duration_ms;
             return o;
           },
           py::arg("tool"), py::arg("agent"), py::arg("task") = "", py::arg("input_json") = py::bytes("{}"),
           py::arg("reason") = "")
      .def("rollback",
           [](ToolService& s, const std::string& id) {
             std::string err;
             bool ok;
             {
               py::gil_scoped_release rel;
               ok = s.rollback(id, err);
             }
             return py::make_tuple(ok, err);
           })
      .def("scan_plugins", &ToolService::scan_plugins)
      .def("tool_count", &ToolService::tool_count)
      .def("grant", [](ToolService& s, const std::string& a, const std::vector<std::string>& c) { s.caps().grant(a, c); })
      .def("revoke",
           [](ToolService& s, const std::string& a, const std::vector<std::string>& c, bool all) {
             return s.caps().revoke(a, c, all);
           },
           py::arg("agent"), py::arg("caps") = std::vector<std::string>{}, py::arg("all") = false)
      .def("register_agent_caps",
           [](ToolService& s, const std::string& a, const std::vector<std::string>& c) { s.caps().register_agent(a, c); })
      .def("agent_caps", [](ToolService& s, const std::string& a) { return s.caps().agent_caps(a); })
      .def("check",
           [](ToolService& s, const std::string& a, const std::string& t) {
             CapCheck c = s.caps().check(a, t);
             py::dict o;
             o["allowed"] = c.allowed;
             o["reason"] = c.reason;
             o["risk"] = c.risk;
             o["missing"] = c.missing;
             return o;
           })
      .def_static("all_capabilities", &CapabilityChecker::all_capabilities)
      .def("audit_verify", [](ToolService& s) {
        py::gil_scoped_release rel;
        return s.audit().verify_chain();
      })
      .def("audit_count", [](ToolService& s) { return s.audit().count(); })
      .def("audit_query",
           [](ToolService& s, const std::string& tool, const std::string& agent, const std::string& since,
              const std::string& until, int limit) { return to_py(s.audit().query(tool, agent, since, until, limit)); },
           py::arg("tool") = "", py::arg("agent") = "", py::arg("since") = "", py::arg("until") = "",
           py::arg("limit") = 100);

  // ---------------------------------------------------------------- memory
  py::class_<MemoryStore>(m, "MemoryStore")
      .def(py::init<const std::string&, const std::string&, const std::string&>())
      .def("push_event", [](MemoryStore& s, py::object ev) { s.operational().push_event(to_json(ev)); })
      .def("recent_events",
           [](MemoryStore& s, int n, const std::string& cat, const std::string& src) {
             return to_py(s.operational().recent(n, cat, src));
           },
           py::arg("count") = 100, py::arg("category") = "", py::arg("source") = "")
      .def("update_metric",
           [](MemoryStore& s, const std::string& k, double v, int64_t ts) { s.operational().update_metric(k, v, ts); })
      .def("get_metric",
           [](MemoryStore& s, const std::string& k) -> py::object {
             double v;
             int64_t ts;
             if (!s.operational().metric(k, v, ts)) return py::none();
             return py::make_tuple(v, ts);
           })
      .def("snapshot", [](MemoryStore& s) { return to_py(s.operational().snapshot()); })
      .def("store_goal", [](MemoryStore& s, py::object g) { s.store_goal(to_json(g)); })
      .def("update_goal", &MemoryStore::update_goal)
      .def("active_goals", [](MemoryStore& s) { return to_py(s.active_goals()); })
      .def("store_task", [](MemoryStore& s, py::object t) { s.store_task(to_json(t)); })
      .def("tasks_for_goal", [](MemoryStore& s, const std::string& g) { return to_py(s.tasks_for_goal(g)); })
      .def("store_tool_call", [](MemoryStore& s, py::object c) { s.store_tool_call(to_json(c)); })
      .def("store_decision", [](MemoryStore& s, py::object d) { s.store_decision(to_json(d)); })
      .def("store_pattern", [](MemoryStore& s, py::object p) { s.store_pattern(to_json(p)); })
      .def("find_pattern",
           [](MemoryStore& s, const std::string& t, double ms) { return to_py(s.find_pattern(t, ms)); },
           py::arg("trigger"), py::arg("min_success_rate") = 0.0)
      .def("update_pattern_stats", &MemoryStore::update_pattern_stats)
      .def("store_agent_state", &MemoryStore::store_agent_state)
      .def("agent_state", [](MemoryStore& s, const std::string& a) { return to_py(s.agent_state(a)); })
      .def("learn_pattern_from_goal", [](MemoryStore& s, const std::string& g) { return to_py(s.learn_pattern_from_goal(g)); })
      .def("tool_sequence_for_goal", [](MemoryStore& s, const std::string& g) { return to_py(s.tool_sequence_for_goal(g)); })
      .def("store_procedure", [](MemoryStore& s, py::object p) { s.store_procedure(to_json(p)); })
      .def("store_incident", [](MemoryStore& s, py::object i) { s.store_incident(to_json(i)); })
      .def("store_config_change", [](MemoryStore& s, py::object c) { s.store_config_change(to_json(c)); })
      .def("semantic_search",
           [](MemoryStore& s, const std::string& q, const std::vector<std::string>& cols, int n, double mr) {
             return to_py(s.semantic_search(q, cols, n, mr));
           },
           py::arg("query"), py::arg("collections") = std::vector<std::string>{}, py::arg("n_results") = 5,
           py::arg("min_relevance") = 0.0)
      .def("add_knowledge", [](MemoryStore& s, py::object k) { s.add_knowledge(to_json(k)); })
      .def("search_knowledge",
           [](MemoryStore& s, const std::string& q, int n, double mr) { return to_py(s.search_knowledge(q, n, mr)); },
           py::arg("query"), py::arg("n_results") = 5, py::arg("min_relevance") = 0.0)
      .def("assemble_context",
           [](MemoryStore& s, const std::string& task, int mt, const std::vector<std::string>& tiers) {
             return to_py(s.assemble_context(task, mt, tiers));
           },
           py::arg("task"), py::arg("max_tokens") = 0, py::arg("tiers") = std::vector<std::string>{})
      .def("migrate",
           [](MemoryStore& s, int64_t ga, int mp, int64_t ca) {
             Json r;
             {
               py::gil_scoped_release rel;
               r = s.migrate(ga, mp, ca);
             }
             return to_py(r);
           },
           py::arg("max_goal_age_s") = 3600, py::arg("max_patterns") = 1000, py::arg("max_call_age_s") = 48 * 3600)
      .def("stats", [](MemoryStore& s) { return to_py(s.stats()); });

  // ---------------------------------------------------------------- planner / llm
  auto pl = m.def_submodule("planner");
  pl.def("classify", &planner::classify);
  pl.def("infer_tools", &planner::infer_tools);
  pl.def("extract_service_name", &planner::extract_service_name);
  pl.def("analyze_steps", &planner::analyze_steps);
  pl.def("decompose", [](const std::string& gid, const std::string& d, const std::string& lvl) {
    return to_py(planner::decompose(gid, d, lvl));
  });
  pl.def("parse_ai_decomposition", [](const std::string& t, const std::string& gid, const std::string& lvl) {
    return to_py(planner::parse_ai_decomposition(t, gid, lvl));
  });
  pl.def("ai_decomposition_prompt", &planner::ai_decomposition_prompt);
  pl.attr("DECOMPOSE_SYSTEM_PROMPT") = std::string(planner::kDecomposeSystemPrompt);

  auto lm = m.def_submodule("llm");
  lm.def("strip_think", &llm::strip_think);
  lm.def("extract_json", [](const std::string& t) -> py::object {
    Json j;
    if (!llm::extract_json(t, j)) return py::none();
    return to_py(j);
  });
  lm.def("parse_tool_calls", [](const std::string& t) { return to_py(llm::parse_tool_calls(t)); });
  lm.def("tools_from_natural_language", [](const std::string& t) { return to_py(llm::tools_from_natural_language(t)); });
  lm.def("parse_clarification", [](const std::string& t) -> py::object {
    std::string q;
    if (!llm::parse_clarification(t, q)) return py::none();
    return py::str(q);
  });
  lm.def("heuristic_calls", [](py::object task) { return to_py(llm::heuristic_calls(to_json(task))); });
  lm.def("explicit_tool_call", [](const std::string& d) -> py::object {
    Json c;
    if (!llm::explicit_tool_call(d, c)) return py::none();
    return to_py(c);
  });
  lm.def("json_to_readable", [](py::object v) { return llm::json_to_readable(to_json(v)); });
  lm.def("summarize_tool_output",
         [](const std::string& tool, py::object out, size_t mc) { return llm::summarize_tool_output(tool, to_json(out), mc); },
         py::arg("tool"), py::arg("output"), py::arg("max_chars") = 1000);
  lm.def("is_done_signal", &llm::is_done_signal);

  // ---------------------------------------------------------------- orchestrator stores
  py::class_<GoalEngine>(m, "GoalEngine")
      .def(py::init<const std::string&>())
      .def("submit",
           [](GoalEngine& g, const std::string& d, int p, const std::string& src, py::object tags,
              const py::bytes& meta) { return to_py(g.submit(d, p, src, to_json(tags), std::string(meta))); },
           py::arg("description"), py::arg("priority") = 5, py::arg("source") = "user", py::arg("tags") = py::list(),
           py::arg("metadata_json") = py::bytes(""))
      .def("goal", [](GoalEngine& g, const std::string& id) { return to_py(g.goal(id)); })
      .def("list",
           [](GoalEngine& g, const std::string& st, int lim, int off) {
             int total = 0;
             Json l = g.list(st, lim, off, total);
             return py::make_tuple(to_py(l), total);
           },
           py::arg("status") = "", py::arg("limit") = 50, py::arg("offset") = 0)
      .def("cancel", &GoalEngine::cancel)
      .def("set_goal_status", &GoalEngine::set_goal_status)
      .def("set_goal_metadata",
           [](GoalEngine& g, const std::string& id, const std::string& k, py::object v) {
             g.set_goal_metadata(id, k, to_json(v));
           })
      .def("add_tasks", [](GoalEngine& g, const std::string& gid, py::object t) { g.add_tasks(gid, to_json(t)); })
      .def("task", [](GoalEngine& g, const std::string& id) { return to_py(g.task(id)); })
      .def("tasks_for_goal", [](GoalEngine& g, const std::string& id) { return to_py(g.tasks_for_goal(id)); })
      .def("update_task", [](GoalEngine& g, py::object t) { g.update_task(to_json(t)); })
      .def("next_tasks", [](GoalEngine& g, int n) { return to_py(g.next_tasks(n)); }, py::arg("max") = 10)
      .def("progress", &GoalEngine::progress)
      .def("phase", &GoalEngine::phase)
      .def("check_completion", &GoalEngine::check_completion)
      .def("add_message", &GoalEngine::add_message)
      .def("messages", [](GoalEngine& g, const std::string& id, int n) { return to_py(g.messages(id, n)); },
           py::arg("goal_id"), py::arg("limit") = 50)
      .def("resume_in_progress", &GoalEngine::resume_in_progress)
      .def("counts", [](GoalEngine& g) { return to_py(g.counts()); })
      .def("pending_goals_without_tasks", [](GoalEngine& g) { return to_py(g.pending_goals_without_tasks()); });

  py::class_<AgentRouter>(m, "AgentRouter")
      .def(py::init<int>(), py::arg("heartbeat_timeout_s") = 15)
      .def("register", [](AgentRouter& r, py::object reg) { r.register_agent(to_json(reg)); })
      .def("unregister", &AgentRouter::unregister)
      .def("heartbeat", &AgentRouter::heartbeat, py::arg("agent_id"), py::arg("status") = "",
           py::arg("task_id") = "")
      .def("list", [](AgentRouter& r) { return to_py(r.list()); })
      .def("route", [](AgentRouter& r, py::object t) { return r.route(to_json(t)); })
      .def("assign", &AgentRouter::assign)
      .def("task_completed", &AgentRouter::task_completed)
      .def("dead_agents", [](AgentRouter& r) { return to_py(r.dead_agents()); })
      .def("healthy_count", &AgentRouter::healthy_count);

  py::class_<ClusterManager>(m, "ClusterManager")
      .def(py::init<int>(), py::arg("timeout_s") = 30)
      .def("register_node", [](ClusterManager& c, py::object n) { c.register_node(to_json(n)); })
      .def("heartbeat", &ClusterManager::heartbeat)
      .def("list", [](ClusterManager& c, bool d) { return to_py(c.list(d)); }, py::arg("include_dead") = false)
      .def("route_least_loaded", &ClusterManager::route_least_loaded)
      .def("prune", &ClusterManager::prune);

  py::class_<Discovery>(m, "Discovery")
      .def(py::init<int>(), py::arg("ttl_s") = 30)
      .def("register_service", &Discovery::register_service)
      .def("heartbeat", &Discovery::heartbeat)
      .def("lookup", [](Discovery& d, const std::string& n) { return to_py(d.lookup(n)); })
      .def("list", [](Discovery& d) { return to_py(d.list()); })
      .def("prune", &Discovery::prune);

  py::class_<DecisionLog>(m, "DecisionLog")
      .def(py::init<size_t>(), py::arg("capacity") = 10000)
      .def("log",
           [](DecisionLog& d, const std::string& ctx, py::object opts, const std::string& ch, const std::string& rs,
              const std::string& lvl, const std::string& model) { return d.log(ctx, to_json(opts), ch, rs, lvl, model); },
           py::arg("context"), py::arg("options"), py::arg("chosen"), py::arg("reasoning"),
           py::arg("intelligence_level") = "", py::arg("model_used") = "")
      .def("update_outcome", &DecisionLog::update_outcome)
      .def("success_rate", &DecisionLog::success_rate, py::arg("context") = "")
      .def("recent", [](DecisionLog& d, int n) { return to_py(d.recent(n)); }, py::arg("n") = 20)
      .def("__len__", &DecisionLog::size);

  py::class_<ResultAggregator>(m, "ResultAggregator")
      .def(py::init<>())
      .def("record", [](ResultAggregator& r, const std::string& g, py::object res) { r.record(g, to_json(res)); })
      .def("results", [](ResultAggregator& r, const std::string& g) { return to_py(r.results(g)); })
      .def("summary", [](ResultAggregator& r, const std::string& g) { return to_py(r.summary(g)); });

  m.def("cron_matches", &cron_matches);
  m.def("cron_valid", &cron_valid);
  py::class_<ScheduleStore>(m, "ScheduleStore")
      .def(py::init<const std::string&>())
      .def("create", &ScheduleStore::create, py::arg("cron_expr"), py::arg("goal_template"), py::arg("priority") = 5)
      .def("list", [](ScheduleStore& s) { return to_py(s.list()); })
      .def("remove", &ScheduleStore::remove)
      .def("due", [](ScheduleStore& s, int64_t now) { return to_py(s.due(now)); });

  // ---------------------------------------------------------------- security / plugin runtime
  m.def("toml_parse", [](const std::string& t) { return to_py(toml_parse(t)); });
  m.def("schema_validate", [](py::object v, py::object schema) { return schema_validate(to_json(v), to_json(schema)); });
  m.def("trigger_check_cron", &trigger_check_cron);
  m.def("trigger_check_file_watch", &trigger_check_file_watch);
  m.def("trigger_check_metric", &trigger_check_metric);
  m.def("trigger_check_log_pattern", &trigger_check_log_pattern);
  py::class_<SecretManager>(m, "SecretManager")
      .def(py::init<const std::string&, int>(), py::arg("path"), py::arg("ttl_s") = 3600)
      .def("load", &SecretManager::load)
      .def("get", [](const SecretManager& s, const std::string& k) -> py::object {
        std::string v;
        if (s.get(k, v)) return py::str(v);
        return py::none();
      })
      .def("get_or_reload", &SecretManager::get_or_reload)
      .def("set", &SecretManager::set)
      .def("wipe", &SecretManager::wipe)
      .def("api_keys", [](SecretManager& s) { return to_py(s.api_keys()); })
      .def("warnings", &SecretManager::warnings)
      .def("__len__", &SecretManager::count);
  auto rule_py = [](const FirewallRule& r) {
    py::dict d;
    d["name"] = r.name; d["action"] = r.action; d["direction"] = r.direction; d["protocol"] = r.protocol;
    d["source"] = r.source; d["destination"] = r.destination; d["interface"] = r.interface;
    d["comment"] = r.comment; d["port"] = r.port; d["port_range"] = py::make_tuple(r.port_lo, r.port_hi);
    d["state"] = r.state;
    return d;
  };
  py::class_<FirewallApplicator>(m, "FirewallApplicator")
      .def(py::init<const std::string&, const std::string&>(), py::arg("config_path"), py::arg("backend") = "auto")
      .def("load_config", [rule_py](const FirewallApplicator& f) {
        std::map<std::string, std::string> pol;
        py::list rules;
        for (auto& r : f.load_config(&pol)) rules.append(rule_py(r));
        return py::make_tuple(rules, pol);
      })
      .def("dry_run", &FirewallApplicator::dry_run)
      .def("setup_commands", &FirewallApplicator::setup_commands)
      .def("apply", [](FirewallApplicator& f, bool dry) { return to_py(f.apply(dry)); }, py::arg("dry_run") = true)
      .def("record_all_applied", [](FirewallApplicator& f) {
        for (auto& r : f.load_config()) f.record_applied(r);
      })
      .def("rollback_commands", &FirewallApplicator::rollback_commands)
      .def("applied_count", &FirewallApplicator::applied_count)
      .def_property_readonly("uses_nftables", &FirewallApplicator::uses_nftables);
  auto trig_py = [](const PluginTrigger& t) {
    py::dict d;
    d["id"] = t.id; d["plugin"] = t.plugin; d["type"] = t.type; d["config"] = to_py(t.config);
    d["enabled"] = t.enabled; d["last_fired"] = t.last_fired;
    return d;
  };
  py::class_<TriggerStore>(m, "TriggerStore")
      .def(py::init<const std::string&>())
      .def("add", [](TriggerStore& s, const std::string& p, const std::string& t, py::object c) { return s.add(p, t, to_json(c)); })
      .def("remove", &TriggerStore::remove)
      .def("set_enabled", &TriggerStore::set_enabled)
      .def("list", [trig_py](const TriggerStore& s) {
        py::list l;
        for (auto& t : s.list()) l.append(trig_py(t));
        return l;
      })
      .def("due", [trig_py](TriggerStore& s, int64_t now, py::object metrics, py::object logs) {
        py::list l;
        for (auto& t : s.due(now, to_json(metrics), to_json(logs))) l.append(trig_py(t));
        return l;
      }, py::arg("now"), py::arg("metrics") = py::dict(), py::arg("log_lines") = py::dict());
  py::class_<PluginWatcher>(m, "PluginWatcher")
      .def(py::init<const std::string&>())
      .def("poll", [](PluginWatcher& w) { return to_py(w.poll()); });
  py::class_<TlsManager>(m, "TlsManager")
      .def(py::init<const std::string&>())
      .def("certs_exist", &TlsManager::certs_exist)
      .def("generate_self_signed", [](TlsManager& t, const std::string& svc, int days) {
        return to_py(t.generate_self_signed(svc, days));
      }, py::arg("service") = "", py::arg("days") = 365)
      .def("verify", [](const TlsManager& t) { return to_py(t.verify()); })
      .def("paths", [](const TlsManager& t) { return to_py(t.paths()); });

  py::class_<EventBus>(m, "EventBus")
      .def(py::init<>())
      .def("subscribe", &EventBus::subscribe, py::arg("pattern"), py::arg("min_severity") = "info",
           py::arg("goal_template") = "", py::arg("priority") = 3)
      .def("unsubscribe", &EventBus::unsubscribe)
      .def("publish", [](EventBus& b, py::object ev) { return to_py(b.publish(to_json(ev))); })
      .def("recent", [](EventBus& b, int n) { return to_py(b.recent(n)); }, py::arg("n") = 20);

  m.def("build_system_prompt",
        [](const std::string& task, const std::string& lvl, py::object tools, py::object pats, int mt) {
          return build_system_prompt(task, lvl, to_json(tools), to_json(pats), mt);
        },
        py::arg("task"), py::arg("level"), py::arg("tools") = py::list(), py::arg("patterns") = py::list(),
        py::arg("max_tokens") = 2048);

  // ---- api-gateway core (gateway.h)
  auto gw = m.def_submodule("gateway", "api-gateway budget ledger, response cache and routing policy");
  py::class_<GwCompletion>(gw, "Completion")
      .def(py::init([](std::string text, int64_t tokens_used, int64_t latency_ms, std::string model_used,
                       int64_t input_tokens, int64_t output_tokens, std::string provider) {
             GwCompletion c;
             c.text = std::move(text); c.tokens_used = tokens_used; c.latency_ms = latency_ms;
             c.model_used = std::move(model_used); c.input_tokens = input_tokens; c.output_tokens = output_tokens;
             c.provider = std::move(provider);
             return c;
           }),
           py::arg("text") = "", py::arg("tokens_used") = 0, py::arg("latency_ms") = 0, py::arg("model_used") = "",
           py::arg("input_tokens") = 0, py::arg("output_tokens") = 0, py::arg("provider") = "")
      .def_readwrite("text", &GwCompletion::text)
      .def_readwrite("tokens_used", &GwCompletion::tokens_used)
      .def_readwrite("latency_ms", &GwCompletion::latency_ms)
      .def_readwrite("model_used", &GwCompletion::model_used)
      .def_readwrite("input_tokens", &GwCompletion::input_tokens)
      .def_readwrite("output_tokens", &GwCompletion::output_tokens)
      .def_readwrite("provider", &GwCompletion::provider);
  py::class_<BudgetLedger>(gw, "BudgetLedger")
      .def(py::init<double, double, const std::string&>(), py::arg("claude_budget") = 100.0,
           py::arg("openai_budget") = 50.0, py::arg("db_path") = ":memory:")
      .def("record", &BudgetLedger::record, py::arg("provider"), py::arg("model"), py::arg("input_tokens"),
           py::arg("output_tokens"), py::arg("tokens_used"), py::arg("cost_usd"), py::arg("agent") = "",
           py::arg("task") = "", py::arg("now") = 0, py::call_guard<py::gil_scoped_release>())
      .def("used", &BudgetLedger::used, py::arg("provider"), py::arg("now") = 0, py::call_guard<py::gil_scoped_release>())
      .def("provider_exceeded", &BudgetLedger::provider_exceeded, py::arg("provider"), py::arg("now") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("exceeded", &BudgetLedger::exceeded, py::arg("now") = 0, py::call_guard<py::gil_scoped_release>())
      .def("status", [](BudgetLedger& b, int64_t now) { return to_py(b.status(now)); }, py::arg("now") = 0)
      .def("usage", [](BudgetLedger& b, const std::string& p, int days, int64_t now) { return to_py(b.usage(p, days, now)); },
           py::arg("provider") = "", py::arg("days") = 30, py::arg("now") = 0)
      .def_property_readonly("claude_budget", &BudgetLedger::claude_budget)
      .def_property_readonly("openai_budget", &BudgetLedger::openai_budget)
      .def_static("month_start", &BudgetLedger::month_start);
  py::class_<ResponseCache>(gw, "ResponseCache")
      .def(py::init<double, size_t>(), py::arg("ttl") = 3600.0, py::arg("max_entries") = 1000)
      .def_static("key", &ResponseCache::key)
      .def("get", &ResponseCache::get, py::arg("key"), py::arg("now") = 0.0)
      .def("put", &ResponseCache::put, py::arg("key"), py::arg("completion"), py::arg("now") = 0.0)
      .def("__len__", &ResponseCache::size)
      .def("clear", &ResponseCache::clear);
  gw.def("select", &gw_select, py::arg("preferred"), py::arg("available"), py::arg("budget"), py::arg("now") = 0,
         py::call_guard<py::gil_scoped_release>());
  gw.def("chain", &gw_chain, py::arg("primary"), py::arg("allow_fallback"));
  gw.def("cost", &gw_cost, py::arg("provider"), py::arg("input_tokens"), py::arg("output_tokens"));
  gw.def("wants_json", &gw_wants_json, py::arg("prompt"), py::arg("system_prompt"));
}
