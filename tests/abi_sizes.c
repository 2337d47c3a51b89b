/* prints sizeof/offsetof of the ABI structs for tests/test_abi.py */
#include <stddef.h>
#include <stdio.h>
#include "../include/sentinel_gpu.h"
int main(void) {
    printf("sg_config %zu\n", sizeof(sg_config));
    printf("sg_flow_rule %zu\n", sizeof(sg_flow_rule));
    printf("sg_degrade_rule %zu\n", sizeof(sg_degrade_rule));
    printf("sg_param_item %zu\n", sizeof(sg_param_item));
    printf("sg_param_rule %zu\n", sizeof(sg_param_rule));
    printf("sg_event %zu\n", sizeof(sg_event));
    printf("sg_metric_node %zu\n", sizeof(sg_metric_node));
    printf("sg_bucket %zu\n", sizeof(sg_bucket));
    printf("sg_node_state %zu\n", sizeof(sg_node_state));
    printf("sg_token_req %zu\n", sizeof(sg_token_req));
    printf("sg_token_result %zu\n", sizeof(sg_token_result));
    printf("sg_param_token_req %zu\n", sizeof(sg_param_token_req));
    printf("ev.aux %zu\n", offsetof(sg_event, aux));
    printf("cfg.cluster_exceed_count %zu\n", offsetof(sg_config, cluster_exceed_count));
    printf("param.items %zu\n", offsetof(sg_param_rule, items));
    printf("cfg.aux_node_capacity %zu\n", offsetof(sg_config, aux_node_capacity));
    printf("sg_event_ext %zu\n", sizeof(sg_event_ext));
    printf("sg_arg %zu\n", sizeof(sg_arg));
    return 0;
}
