// code_object.h — resource figures of the kernels in an AMDGPU code object (ELF), read from its metadata note.
//
// The run-time render kernels are built by hipRTC; what the register allocator did to them (VGPRs, SGPRs, scratch,
// spilled registers) is in the code object's NT_AMDGPU_METADATA note (msgpack, "amdhsa.kernels") and the compiler's
// identity in its .comment section.  No device needed.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace rt {

struct KernelMeta {
  std::string name;
  int32_t vgprs = -1, agprs = -1, sgprs = -1;   // per lane (VGPR/AGPR) and per wave (SGPR) counts
  int32_t scratch = -1;                         // private segment bytes per lane (spilled registers live there)
  int32_t vgpr_spills = -1, sgpr_spills = -1;   // registers the allocator spilled (SGPRs: to VGPR lanes or scratch)
  int32_t lds = -1;                             // static LDS bytes
};

// Parses every kernel's figures out of the ELF code object `co`; *compiler (if non-null) receives the first
// "clang version" line of its .comment section ("" if none).  False if `co` is not an AMDGPU ELF with a metadata note.
bool code_object_kernels(const std::vector<char> &co, std::vector<KernelMeta> *out, std::string *compiler);

// The figures of kernel `name` in `co` (false if absent)
bool code_object_kernel(const std::vector<char> &co, const std::string &name, KernelMeta *out, std::string *compiler);

}  // namespace rt
