conditions:
- lastHeartbeatTime: {{ Now }}
  lastTransitionTime: {{ StartTime }}
  message: kubelet is posting ready status (kwok on MI355X)
  reason: KubeletReady
  status: "True"
  type: Ready
- lastHeartbeatTime: {{ Now }}
  lastTransitionTime: {{ StartTime }}
  message: kubelet has sufficient memory available
  reason: KubeletHasSufficientMemory
  status: "False"
  type: MemoryPressure
- lastHeartbeatTime: {{ Now }}
  lastTransitionTime: {{ StartTime }}
  message: kubelet has no disk pressure
  reason: KubeletHasNoDiskPressure
  status: "False"
  type: DiskPressure
- lastHeartbeatTime: {{ Now }}
  lastTransitionTime: {{ StartTime }}
  message: kubelet has sufficient PID available
  reason: KubeletHasSufficientPID
  status: "False"
  type: PIDPressure
- lastHeartbeatTime: {{ Now }}
  lastTransitionTime: {{ StartTime }}
  message: node {{ NodeIP }} has a route
  reason: RouteCreated
  status: "False"
  type: NetworkUnavailable
- lastHeartbeatTime: {{ Now }}
  lastTransitionTime: {{ StartTime }}
  message: kwok fake kubelet
  reason: KwokReady
  status: "True"
  type: example.com/KwokReady
