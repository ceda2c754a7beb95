EDITS = [("cloudsc_place.hip",
"""    } else {
      for (int q = 0; q < n; q++) drop(cf[members[q]], bytes[q]);
    }
  }
  for (auto& sp : spacers) drop(sp.first, sp.second);""",
"""    } else {
      for (int q = 0; q < n; q++) held.push_back({cf[members[q]], bytes[q]});
    }
  }
  for (auto& sp : spacers) drop(sp.first, sp.second);""")]
