// gojson.h -- Go 1.19 encoding/json.Marshal of the reference's message structs.
//
// digest() hashes json.Marshal(obj) (pbft/consensus/pbft_impl.go:235-243), so
// the batch verifier must reproduce Go's bytes exactly to hash the same
// preimages: struct field order and tags of pbft/consensus/pbft_msg_types.go:3-38,
// compact output, decimal int64, the embedded MsgType as "msgType", nil
// *RequestMsg as null, and encodeState.string(escapeHTML=true) escaping.
#pragma once
#include <cstdint>
#include <vector>

#include "gojson_enc.h"

namespace pbftv {
namespace gojson {

void append_string(std::vector<uint8_t>& out, const uint8_t* s, uint64_t n);
void append_int(std::vector<uint8_t>& out, int64_t v);

// RequestMsg (pbft_msg_types.go:3-8)
void append_request(std::vector<uint8_t>& out, int64_t timestamp, const uint8_t* client_id, uint64_t client_id_len,
                    const uint8_t* operation, uint64_t operation_len, int64_t sequence_id);
// VoteMsg (pbft_msg_types.go:25-31)
void append_vote(std::vector<uint8_t>& out, int64_t view_id, int64_t sequence_id, const uint8_t* digest,
                 uint64_t digest_len, const uint8_t* node_id, uint64_t node_id_len, int64_t msg_type);
// signed VoteMsg wire encoding: VoteMsg + "signature":<base64 | null>
void append_vote_signed(std::vector<uint8_t>& out, int64_t view_id, int64_t sequence_id, const uint8_t* digest,
                        uint64_t digest_len, const uint8_t* node_id, uint64_t node_id_len, int64_t msg_type,
                        const uint8_t* sig, uint64_t sig_len, bool sig_nil);
// ReplyMsg (pbft_msg_types.go:10-16)
void append_reply(std::vector<uint8_t>& out, int64_t view_id, int64_t timestamp, const uint8_t* client_id,
                  uint64_t client_id_len, const uint8_t* node_id, uint64_t node_id_len, const uint8_t* result,
                  uint64_t result_len);
// PrePrepareMsg (pbft_msg_types.go:18-23)
void append_preprepare(std::vector<uint8_t>& out, int64_t view_id, int64_t sequence_id, const uint8_t* digest,
                       uint64_t digest_len, bool has_request, int64_t req_timestamp, const uint8_t* req_client_id,
                       uint64_t req_client_id_len, const uint8_t* req_operation, uint64_t req_operation_len,
                       int64_t req_sequence_id);

// signed wire encodings of the other three messages (gojson_enc.h)
void append_request_signed(std::vector<uint8_t>& out, int64_t timestamp, const uint8_t* client_id,
                           uint64_t client_id_len, const uint8_t* operation, uint64_t operation_len,
                           int64_t sequence_id, const SigField& sig);
void append_reply_signed(std::vector<uint8_t>& out, int64_t view_id, int64_t timestamp, const uint8_t* client_id,
                         uint64_t client_id_len, const uint8_t* node_id, uint64_t node_id_len, const uint8_t* result,
                         uint64_t result_len, const SigField& sig);
void append_preprepare_signed(std::vector<uint8_t>& out, int64_t view_id, int64_t sequence_id, const uint8_t* digest,
                              uint64_t digest_len, bool has_request, int64_t req_timestamp,
                              const uint8_t* req_client_id, uint64_t req_client_id_len, const uint8_t* req_operation,
                              uint64_t req_operation_len, int64_t req_sequence_id, const SigField& req_sig,
                              const SigField& sig);

}  // namespace gojson
}  // namespace pbftv
