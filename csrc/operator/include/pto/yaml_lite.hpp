// A small YAML subset reader (block mappings / sequences, plain + quoted scalars,
// flow sequences and flow mappings of scalars, comments) -> Json.
//
// Enough for the operator's init-container template (the reference's Go template
// pkg/common/config/config.go:9-34, overridable from /etc/config/initContainer.yaml)
// and for the simple PyTorchJob manifests under examples/.  Not a general YAML
// implementation: no anchors, tags, multi-documents or block scalars.
#pragma once

#include <string>

#include "pto/json.hpp"

namespace pto {

Json yaml_parse(const std::string& text);  // throws JsonError on malformed input

// Go text/template subset: replaces {{.Key}} with values[Key].
std::string render_template(const std::string& tmpl,
                            const std::vector<std::pair<std::string, std::string>>& values);

}  // namespace pto
