conditions:
- lastHeartbeatTime: {{ Now }}
  lastTransitionTime: {{ StartTime }}
  reason: KubeletReady
  status: "True"
  type: Ready
